#!/bin/bash
# A/B the variants/*.so on the physical HBM-tile decoder (GPU box), two rounds:
# DVB-S2-profile config 5 at 1.0 dB and wimax_2304_0.5 forced to HBM tiles at 0 dB.
OUT=gpurun_out/abphys
mkdir -p $OUT
one() {
  lib=$1; tag=$2; shift 2
  name=$(basename $lib .so)
  LDPC_HIP_LIB=$lib timeout -k 10 200 python bench.py --mode physical --steps 3 --warmup 1 --cpu-seconds 0 "$@" > $OUT/${name}_$tag.log 2>&1 || { echo "FAIL $name $tag"; tail -3 $OUT/${name}_$tag.log; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/${name}_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name $tag'.ljust(22), round(d['value']), 'cw/s ', r['kernel'], round(r['avg_launch_ms'],3), 'ms x', r['launches'], 'frac', round(r.get('frac') or 0,3), 'iters', round(d['avg_iters'],2))"
}
for round in 1 2; do
  for lib in variants/*.so; do
    one $lib dvbs2 --code dvbs2_profile_64800_0.5 --snr 1.0 --frames 8192 || exit 1
    one $lib w2304hbm --phys-hbm --code wimax_2304_0.5 --snr 0.0 --frames 65536 --chunk 16384 || exit 1
  done
done
