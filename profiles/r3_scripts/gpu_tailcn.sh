#!/bin/bash
# split-path CN at the 3 dB tail's size (1,152 frames = 18 tiles, 1 dB, T=50):
# cn_kernel vs cn_row_kernel 16x40 (LDPC_CN_ROW16=1), per-kernel times from rocprofv3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tailcn}; mkdir -p $O
B="--frames ${FR:-1152} --split --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for v in ${VARS:-cn row16}; do
  E=LDPC_CN_ROW16=0; [ $v = row16 ] && E=LDPC_CN_ROW16=1
  export $E
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py $B > $O/$v.json 2> $O/$v.err || { tail $O/$v.err; exit 1; }
  python3 - $O/$v <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:6]: print(' ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms avg')
PY
  echo "$v $(python tools/bench_summary.py $O/$v.json)"
done
