#!/bin/bash
# tile8 / tile_sub after the branch-free hop: parity tests, A/B bench, timers.
set -o pipefail
O=gpurun_out/${TAG:-t8c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_config3.py -x -v --timeout 300 --timeout-method thread > $O/t1.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/t1.log | tail -30; tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
B="--frames 16384 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for v in new old; do
  E=""; [ $v = old ] && E="LDPC_TILE8=0"
  env $E timeout -k 10 300 python -u bench.py $B > $O/$v.json 2> $O/$v.err && python tools/bench_summary.py $O/$v.json || { tail $O/$v.err; exit 1; }
done
timeout -k 10 300 python -u bench.py $B --code wimax_2304_0.75A > $O/r34_new.json 2> $O/r34_new.err && python tools/bench_summary.py $O/r34_new.json || exit 1
LDPC_HIP_LIB=variants/t8diag.so timeout -k 10 200 python -u bench.py --frames 4096 --steps 1 --warmup 0 --cpu-seconds 0 --extra-snr= --phys-steps 0 > $O/timers.log 2>&1 || { tail -20 $O/timers.log; exit 1; }
grep "^T8 b=0" $O/timers.log | sort -t= -k3 -n | head -16
