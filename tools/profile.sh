#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel trace + stats of the bench
# workload, then one PMC pass per TCC counter group (FETCH_SIZE and WRITE_SIZE
# cannot share a pass on gfx950).  Outputs under gpurun_out/$TAG.
# usage: tools/profile.sh TAG [bench args...]
set -e
TAG=${1:-prof}; shift || true
ARGS=${@:---steps 1 --warmup 1 --cpu-seconds 0}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1
echo done
