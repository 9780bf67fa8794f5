#!/bin/bash
# edge-path tests, then one-frame..8-frame decode latency: base vs synrow variants
set -o pipefail
O=gpurun_out/${TAG:-synrow}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_00_fork.py tests/test_gpu_edge.py tests/test_gpu_smallcols.py tests/test_gpu_dropin.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for round in 1 2; do for v in "$@"; do
  LDPC_HIP_LIB=variants/$v.so CODE=${CODE:-wimax_2304_0.5} BS=1,4,8 timeout -k 10 200 python -u tools/probe_small.py - > $O/${v}_$round.jsonl 2> $O/${v}_$round.err || { tail $O/${v}_$round.err; exit 1; }
  python -c "
import json
for l in open('$O/${v}_$round.jsonl'): d=json.loads(l); print('$v r$round', d['B'], d['ms_per_call'])"
done; done
