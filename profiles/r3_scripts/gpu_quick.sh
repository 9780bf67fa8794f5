#!/bin/bash
# quick GPU check: selected tests (TESTS, pytest -k expression over the gpu suite) then the short point bench.
set -o pipefail
O=gpurun_out/${TAG:-quick}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:+-k "$TESTS"} > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
LDPC_TAIL_LOG=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-seconds 0 --phys-steps 0 ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
