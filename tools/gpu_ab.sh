#!/bin/bash
# Reusable A/B on the GPU box: bench.py with the flags in $B once per variant
# in $LIBS, in the order given, $REPS times.  A variant is a library name
# (variants/<name>.so built by tools/build_variants.sh; "main" = the in-tree
# libldpc_hip.so), optionally followed by ":VAR=value[,VAR=value]" environment
# settings for that run (e.g. "main:LDPC_LPT=0").
# usage: TAG=ab LIBS="base col16 main:LDPC_LPT=0" B="--frames 16384 --steps 1 ..." REPS=2 bash tools/gpu_ab.sh
set -o pipefail
O=gpurun_out/${TAG:-ab}; mkdir -p $O
for rep in $(seq 1 ${REPS:-1}); do
  for spec in $LIBS; do
    v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
    name=$(echo "$spec" | tr ':=,' '___')
    if [ "$v" = main ]; then lib=""; else lib="LDPC_HIP_LIB=$PWD/variants/$v.so"; fi
    env $lib $(echo "$envs" | tr ',' ' ') timeout -k 10 ${AB_TIMEOUT:-300} python -u bench.py $B > $O/${name}_$rep.json 2> $O/${name}_$rep.err || { tail -20 $O/${name}_$rep.err; exit 1; }
    echo "$spec#$rep $(python tools/bench_summary.py $O/${name}_$rep.json)"
  done
done
