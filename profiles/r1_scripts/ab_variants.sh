#!/bin/bash
# A/B the library variants in variants/*.so on one box (compile-time switches), two interleaved rounds.
for round in 1 2; do
  for lib in variants/*.so; do
    name=$(basename $lib .so)
    LDPC_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/ab_${name}_$round.log 2>&1 || { echo "FAIL $lib"; continue; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab_${name}_$round.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name r$round'.ljust(14), round(d['value']), 'cw/s  cn', round(r['avg_launch_ms'],3), 'ms  vn', round(d['decode_roofline']['vn_ms']/r['launches'],3))"
  done
done
