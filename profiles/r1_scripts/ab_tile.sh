#!/bin/bash
# A/B the variants/*.so on the tile-resident decoder (GPU box): static schedule,
# one tile per CU (16,384 frames), wimax_576_0.5, 50 iterations, 0 dB; two rounds.
FR=${FRAMES:-16384}
mkdir -p gpurun_out/abtile
for round in 1 2; do
  for lib in variants/*.so; do
    name=$(basename $lib .so)
    LDPC_HIP_LIB=$lib timeout -k 10 120 python bench.py --schedule static --frames $FR --steps 2 --warmup 1 --cpu-seconds 0 "$@" > gpurun_out/abtile/${name}_$round.log 2>&1 || { echo "FAIL $name"; tail -3 gpurun_out/abtile/${name}_$round.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/abtile/${name}_$round.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name r$round'.ljust(20), round(d['value']), 'cw/s ', r['kernel'], round(r['avg_launch_ms'],2), 'ms/launch frac', round(r['frac'],3), 'iters', round(d['avg_iters'],2))"
  done
done
