#!/bin/bash
# edge path on every code: full GPU suite, then latency of small batches on wimax_576_0.5 and 2304 r1/2, r3/4A
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-edge2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for code in wimax_576_0.5 wimax_2304_0.5 wimax_2304_0.75A; do
  CODE=$code BS=1,8,16,32,64 timeout -k 10 300 python -u tools/probe_small.py - LDPC_EDGE_FRAMES=0 > $O/lat_$code.jsonl 2> $O/lat_$code.err || { tail $O/lat_$code.err; exit 1; }
  cat $O/lat_$code.jsonl
done
