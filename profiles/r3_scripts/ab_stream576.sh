#!/bin/bash
# A/B of library variants on the 64-frame streaming tile kernel (wimax_576_0.5,
# 65,536 frames, 2 and 3 dB) and the 2304 r1/2 3 dB whole point.  usage: TAG=x tools/ab_stream576.sh name...
set -o pipefail
O=gpurun_out/${TAG:-ab576s}; mkdir -p $O
for round in 1 2; do
  for name in "$@"; do
    lib=variants/$name.so
    for cfg in a2 a3 p3; do
      case $cfg in
        a2) A="--code wimax_576_0.5 --frames 65536 --snr 2.0 --schedule stream --steps 2 --warmup 1 --extra-snr= --point-snr=";;
        a3) A="--code wimax_576_0.5 --frames 65536 --snr 3.0 --schedule stream --steps 2 --warmup 1 --extra-snr= --point-snr=";;
        p3) A="--frames 4096 --steps 1 --warmup 0 --extra-snr=";;
      esac
      LDPC_HIP_LIB=$lib timeout -k 10 200 python bench.py $A --cpu-seconds 0 --phys-steps 0 > $O/${name}_${cfg}_$round.json 2> $O/${name}_${cfg}_$round.err || { echo "FAIL $name $cfg"; tail -5 $O/${name}_${cfg}_$round.err; exit 1; }
      python -c "
import json; d=json.loads(open('$O/${name}_${cfg}_$round.json').read().strip().splitlines()[-1])
pts=[(p['snr_db'],p.get('scope'),round(p['value'])) for p in d.get('snr_points',[])]
print('$name $cfg r$round'.ljust(18), round(d['value']), 'cw/s', round(d['ms_per_step'],1), 'ms', pts)"
    done
  done
done
