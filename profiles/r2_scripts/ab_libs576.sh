#!/bin/bash
# A/B library variants (variants/<name>.so) on the config-2 decode
# (wimax_576_0.5, 0 dB, 65,536 frames, static); two interleaved rounds.
# usage: TAG=x tools/ab_libs576.sh name1 name2 ...
set -o pipefail
O=gpurun_out/${TAG:-ab576}; mkdir -p $O
for round in 1 2; do
  for name in "$@"; do
    LDPC_HIP_LIB=variants/$name.so timeout -k 10 200 python bench.py --code wimax_576_0.5 --snr 0.0 --frames 65536 --steps 2 --warmup 1 --cpu-seconds 0 --extra-snr= > $O/${name}_$round.json 2> $O/${name}_$round.err || { echo "FAIL $name"; exit 1; }
    python -c "
import json; d=json.loads(open('$O/${name}_$round.json').read().strip().splitlines()[-1])
print('$name r$round'.ljust(12), round(d['value']), 'cw/s', round(d['roofline']['avg_launch_ms'],2), 'ms/launch', round(d['roofline']['frac'],4))"
  done
done
