#!/bin/bash
# A/B an environment knob on one box: tools/ab_env.sh VAR v1 v2 ... (two interleaved rounds)
VAR=$1; shift
for round in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 120 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/abenv_${VAR}_${v}_$round.log 2>&1 || echo "FAIL $v"
  done
done
echo done
