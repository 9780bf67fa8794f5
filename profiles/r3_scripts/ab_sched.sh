#!/bin/bash
# A/B of library variants (variants/<name>.so): static 1 dB wimax_2304_0.5 (16,384 frames),
# static 1 dB wimax_2304_0.75A (tile8, 16,384 frames), the 3 dB streaming step; two rounds.
set -o pipefail
O=gpurun_out/${TAG:-absched}; mkdir -p $O
for round in 1 2; do
  for name in "$@"; do
    for cfg in h34 h12 s3; do
      case $cfg in
        h12) A="--frames 16384 --steps 1 --warmup 1 --extra-snr= --point-snr=";;
        h34) A="--code wimax_2304_0.75A --frames 16384 --steps 1 --warmup 1 --extra-snr= --point-snr=";;
        s3) A="--frames 32768 --steps 1 --warmup 0 --snr 3.0 --schedule stream --chunk 8192 --extra-snr= --point-snr=";;
      esac
      LDPC_HIP_LIB=variants/$name.so timeout -k 10 200 python bench.py $A --cpu-seconds 0 --phys-steps 0 --dropin-calls 0 > $O/${name}_${cfg}_$round.json 2> $O/${name}_${cfg}_$round.err || { echo "FAIL $name $cfg"; tail -5 $O/${name}_${cfg}_$round.err; exit 1; }
      python -c "
import json; d=json.loads(open('$O/${name}_${cfg}_$round.json').read().strip().splitlines()[-1])
print('$name $cfg r$round'.ljust(22), round(d['value']), 'cw/s', round(d['ms_per_step'],1), 'ms', round(d['roofline'].get('frac') or 0,4), d['roofline'].get('kernel'))"
    done
  done
done
