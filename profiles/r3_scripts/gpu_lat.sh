#!/bin/bash
# one-frame decode() latency on the all-zero codeword (LLR mean -2 ~1 dB, -4, -8 ~3 dB) + trace at mean -4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-lat}; mkdir -p $O
for mean in -2.0 -4.0 -8.0; do
  MEAN=$mean BS=1 timeout -k 10 200 python -u tools/probe_small.py - >> $O/lat.jsonl 2>> $O/lat.err || { tail $O/lat.err; exit 1; }
done
cat $O/lat.jsonl
MEAN=-4.0 BS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/probe_small.py - > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python3 - $O <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/trace/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,3), 'ms')
PY
