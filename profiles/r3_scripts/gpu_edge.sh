#!/bin/bash
# few-frame edge path: its GPU tests, the small-batch suites it now serves, latency vs the frame-per-lane path
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-edge}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_00_fork.py tests/test_gpu_edge.py tests/test_gpu_smallcols.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
BS=1,2,4,8,16,64 timeout -k 10 300 python -u tools/probe_small.py - LDPC_EDGE_FRAMES=0 > $O/lat.jsonl 2> $O/lat.err || { tail $O/lat.err; exit 1; }
cat $O/lat.jsonl
BS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/probe_small.py - > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
python3 - $O <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/trace/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms')
PY
