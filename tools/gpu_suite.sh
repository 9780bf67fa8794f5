#!/bin/bash
# Reusable GPU-box check: the -m gpu suite (or the test files given in $TESTS),
# then smoke(), then (if BENCH is set) one bench.py line with $BENCH's flags.
# Usage on the box: TAG=r4a TESTS="tests/test_gpu_decoders.py" BENCH="--steps 3" bash tools/gpu_suite.sh
set -o pipefail
O=gpurun_out/${TAG:-suite}; mkdir -p $O
T=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $T -m gpu -x -v --timeout ${CASE_TIMEOUT:-300} --timeout-method thread \
    --durations=15 > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/tests.log | tail -40; tail -60 $O/tests.log; exit 1; }
tail -20 $O/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -n "$BENCH" ]; then
    timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py $BENCH > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
    python tools/bench_summary.py $O/bench.json
fi
