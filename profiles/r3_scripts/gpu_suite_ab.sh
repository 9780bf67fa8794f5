#!/bin/bash
# full -m gpu suite (quiet), then tools/ab_3db.sh over the given variants
set -o pipefail
O=gpurun_out/${TAG:-suite_ab}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
TAG=${TAG:-suite_ab}_ab bash tools/ab_3db.sh "$@"
