#!/bin/bash
# A/B of library variants on both 2304 codes: TAG=x tools/gpu_t8f.sh lib1 lib2 ... (lib = variants/<name>.so or 'default')
set -o pipefail
O=gpurun_out/${TAG:-t8f}; mkdir -p $O
B="--frames 16384 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for code in ${CODES:-wimax_2304_0.75A wimax_2304_0.5}; do for v in "$@"; do
  L=""; [ $v != default ] && L="LDPC_HIP_LIB=variants/$v.so"
  env $L timeout -k 10 300 python -u bench.py $B --code $code > $O/${code}_$v.json 2> $O/${code}_$v.err || { tail $O/${code}_$v.err; exit 1; }
  echo "$code $v $(python tools/bench_summary.py $O/${code}_$v.json)"
done; done
