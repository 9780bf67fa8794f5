#!/bin/bash
# A/B on three lines (1 dB headline, r3/4 at 1 dB, 576 at 1 dB) + the 3 dB stream step; LIBS as gpu_ab.sh
set -o pipefail
O=gpurun_out/${TAG:-ab3}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TFILES:-tests/test_gpu_tile.py} -x -q --timeout 300 --timeout-method thread -k "$TESTS" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
  tail -1 $O/t.log
fi
B="--steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for v in ${LIBS:-base new}; do
  E=""; [ $v != new ] && E="LDPC_HIP_LIB=variants/$v.so"
  for line in "r12:--frames 16384" "r34:--frames 16384 --code wimax_2304_0.75A" "w576:--code wimax_576_0.5" "s3:--snr 3.0 --schedule stream --chunk 8192 --frames 32768"; do
    n=${line%%:*}; a=${line#*:}
    env $E timeout -k 10 300 python -u bench.py $B $a > $O/${v}_$n.json 2> $O/${v}_$n.err || { tail $O/${v}_$n.err; exit 1; }
    echo "$v $n $(python tools/bench_summary.py $O/${v}_$n.json)"
  done
done
