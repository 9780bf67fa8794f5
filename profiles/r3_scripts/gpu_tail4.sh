#!/bin/bash
# 3 dB streaming step: compaction threshold A/B (LDPC_COMPACT_AT eighths) with the tail log
set -o pipefail
O=gpurun_out/${TAG:-tail4}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mc.py -x -q --timeout 300 --timeout-method thread -k "stream" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
S="--snr 3.0 --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
for v in ${VARS:-4 6 8}; do
  LDPC_TAIL_LOG=1 LDPC_COMPACT_AT=$v timeout -k 10 300 python -u bench.py $S > $O/s3_$v.json 2> $O/s3_$v.err || { tail $O/s3_$v.err; exit 1; }
  echo "3dB at=$v $(python tools/bench_summary.py $O/s3_$v.json)"
done
