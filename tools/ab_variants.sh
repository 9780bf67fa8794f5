#!/bin/bash
# A/B the library variants in variants/*.so on one box, two interleaved rounds.
for round in 1 2; do
  for lib in variants/*.so; do
    LDPC_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/ab_$(basename $lib .so)_$round.log 2>&1 || echo "FAIL $lib"
  done
done
echo done
