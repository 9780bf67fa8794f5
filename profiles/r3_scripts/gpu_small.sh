#!/bin/bash
# small-batch decode latency variants + a kernel trace of B=1 (default policy)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-small}; mkdir -p $O
timeout -k 10 300 python -u tools/probe_small.py - LDPC_CN_ROW16=1 ${EXTRA_VARS} > $O/lat.jsonl 2> $O/lat.err || { tail $O/lat.err; exit 1; }
cat $O/lat.jsonl
BS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/probe_small.py - > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python3 - $O <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/trace/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms')
PY
