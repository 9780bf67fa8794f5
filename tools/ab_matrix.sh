#!/bin/bash
# variants x LDS pads, two rounds
for round in 1 2; do
  for lib in variants/*.so; do
    for pad in 0 34000 74000; do
      LDPC_HIP_LIB=$lib LDPC_CN_LDS_PAD=$pad timeout -k 10 120 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/abm_$(basename $lib .so)_p${pad}_$round.log 2>&1 || echo "FAIL $lib $pad"
    done
  done
done
echo done
