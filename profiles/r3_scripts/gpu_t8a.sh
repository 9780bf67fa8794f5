#!/bin/bash
# tile8 first light: targeted parity tests, then headline A/B (tile8 vs LDPC_TILE8=0) and r3/4.
set -o pipefail
O=gpurun_out/${TAG:-t8a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_config3.py -x -v --timeout 300 --timeout-method thread > $O/t1.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/t1.log | tail -30; tail -40 $O/t1.log; exit 1; }
tail -2 $O/t1.log
B="--frames 16384 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
timeout -k 10 300 python -u bench.py $B > $O/new.json 2> $O/new.err && python tools/bench_summary.py $O/new.json || { tail $O/new.err; exit 1; }
LDPC_TILE8=0 timeout -k 10 300 python -u bench.py $B > $O/old.json 2> $O/old.err && python tools/bench_summary.py $O/old.json || exit 1
timeout -k 10 300 python -u bench.py $B --code wimax_2304_0.75A > $O/r34_new.json 2> $O/r34_new.err && python tools/bench_summary.py $O/r34_new.json || { tail $O/r34_new.err; exit 1; }
LDPC_TILE8=0 timeout -k 10 300 python -u bench.py $B --code wimax_2304_0.75A > $O/r34_old.json 2> $O/r34_old.err && python tools/bench_summary.py $O/r34_old.json || exit 1
