#!/bin/bash
# A/B on the 2304 r1/2 streaming points: 3 dB one 32,768-frame step (8,192 slots) and
# the whole 262,144-frame 3 dB point; variants name[:ENV=VAL] (variants/<name>.so).
# usage: TAG=x tools/ab_3db.sh old new new:LDPC_CN_ROW16=16
set -o pipefail
O=gpurun_out/${TAG:-ab3db}; mkdir -p $O
for round in 1 2; do
  for v in "$@"; do
    name=${v%%:*}; env=""; [ "$v" != "$name" ] && env=${v#*:}
    tagv=$(echo "$v" | tr ':=' '__')
    A="--frames 32768 --steps 1 --warmup 0 --extra-snr=3.0 --point-snr=3.0 --cpu-seconds 0 --phys-steps 0"
    env LDPC_HIP_LIB=variants/$name.so $env timeout -k 10 200 python bench.py $A > $O/${tagv}_$round.json 2> $O/${tagv}_$round.err || { echo "FAIL $v"; tail -5 $O/${tagv}_$round.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/${tagv}_$round.json').read().strip().splitlines()[-1])
print('$v r$round'.ljust(34), [(p['snr_db'],p.get('scope'),round(p['value']),round(p['ms'])) for p in d.get('snr_points',[])])"
  done
done
