#!/bin/bash
# 3 dB streaming tail: default vs cn_row16 forced; tile8 (r1/2 opt-in) vs tile_sub; r3/4 tile8.
set -o pipefail
O=gpurun_out/${TAG:-t8h}; mkdir -p $O
S="--snr 3.0 --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for v in def row16 def2 row16b; do
  E=""; case $v in row16*) E="LDPC_CN_ROW16=1";; esac
  env $E timeout -k 10 300 python -u bench.py $S > $O/s3_$v.json 2> $O/s3_$v.err || { tail $O/s3_$v.err; exit 1; }
  echo "3dB $v $(python tools/bench_summary.py $O/s3_$v.json)"
done
B="--frames 16384 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for v in t8 sub; do
  E=""; [ $v = t8 ] && E="LDPC_TILE8=1"
  env $E timeout -k 10 300 python -u bench.py $B > $O/h_$v.json 2> $O/h_$v.err || { tail $O/h_$v.err; exit 1; }
  echo "r12 $v $(python tools/bench_summary.py $O/h_$v.json)"
done
timeout -k 10 300 python -u bench.py $B --code wimax_2304_0.75A > $O/r34.json 2> $O/r34.err && echo "r34 $(python tools/bench_summary.py $O/r34.json)"
