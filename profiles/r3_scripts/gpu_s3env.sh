#!/bin/bash
# 3 dB streaming step under environment variants: VARS="name:ENV=val,ENV2=val ..." ("def" = none)
set -o pipefail
O=gpurun_out/${TAG:-s3env}; mkdir -p $O
S="--snr 3.0 --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for r in $(seq ${ROUNDS:-1}); do for v in ${VARS:-def}; do
  n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=$(echo ${v#*:} | tr ',' ' ')
  env $e timeout -k 10 300 python -u bench.py $S > $O/${n}_$r.json 2> $O/${n}_$r.err || { tail $O/${n}_$r.err; exit 1; }
  echo "$n.$r $(python tools/bench_summary.py $O/${n}_$r.json)"
done; done
