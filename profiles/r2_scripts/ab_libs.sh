#!/bin/bash
# A/B library variants (variants/<name>.so) on one box: headline static decode
# (1 dB, 16,384 frames) and the streaming schedule at 2 dB with 8,192 and 4,096
# slots; two interleaved rounds.  usage: TAG=x tools/ab_libs.sh name1 name2 ...
set -o pipefail
O=gpurun_out/${TAG:-ab}; mkdir -p $O
for round in 1 2; do
  for name in "$@"; do
    lib=variants/$name.so
    for cfg in ${CFGS:-s1 t2a t2b}; do
      case $cfg in
        s1) A="--frames 16384 --steps 1 --warmup 1";;
        t2a) A="--snr 2.0 --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 0";;
        t2b) A="--snr 2.0 --schedule stream --chunk 4096 --frames 16384 --steps 1 --warmup 0";;
      esac
      LDPC_HIP_LIB=$lib timeout -k 10 200 python bench.py $A --cpu-seconds 0 --extra-snr= > $O/${name}_${cfg}_$round.json 2> $O/${name}_${cfg}_$round.err || { echo "FAIL $name $cfg"; exit 1; }
      python -c "
import json; d=json.loads(open('$O/${name}_${cfg}_$round.json').read().strip().splitlines()[-1])
print('$name $cfg r$round'.ljust(18), round(d['value']), 'cw/s', round(d['ms_per_step'],1), 'ms', round(d['roofline'].get('frac') or 0,4))"
    done
  done
done
