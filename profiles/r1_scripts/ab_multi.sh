#!/bin/bash
# A/B the variants/*.so over several workloads (GPU box), two rounds:
#   tile    wimax_576_0.5, tile-resident decoder, 16,384 frames, 50 it, 0 dB
#   split   the same through the per-iteration CN/VN launches
#   c3s     wimax_2304_0.5, static chunk of 4,096 frames, 50 it, 0 dB
#   c3t     wimax_2304_0.5, streaming, 65,536 frames through 16,384 slots, 3 dB
OUT=gpurun_out/abmulti
mkdir -p $OUT
one() {
  lib=$1; tag=$2; shift 2
  name=$(basename $lib .so)
  LDPC_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 "$@" > $OUT/${name}_$tag.log 2>&1 || { echo "FAIL $name $tag"; tail -3 $OUT/${name}_$tag.log; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/${name}_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name $tag'.ljust(22), round(d['value']), 'cw/s ', r['kernel'], round(r['avg_launch_ms'],2), 'ms/launch frac', round(r['frac'],3), 'iters', round(d['avg_iters'],2))"
}
for round in 1 2; do
  for lib in variants/*.so; do
    one $lib tile --schedule static --frames 16384 || exit 1
    one $lib split --schedule static --split --frames 16384 || exit 1
    one $lib c3s --code wimax_2304_0.5 --schedule static --frames 4096 --snr 0 || exit 1
    one $lib c3t --code wimax_2304_0.5 --frames 65536 --chunk 16384 --snr 3.0 || exit 1
  done
done
