#!/bin/bash
# Round profile of the headline (tile-resident decoder) on the GPU box:
#   trace       rocprofv3 --kernel-trace --stats of the default bench
#   pmc_fetch   FETCH_SIZE of the same; pmc_fetch_split: FETCH_SIZE of the split
#               path (vn_kernel reads each message exactly once: re-derives the
#               gfx950 FETCH_SIZE correction factor, MI355X_MICROARCH.md §HBM)
#   pmc_write   WRITE_SIZE
# usage: tools/profile_tile.sh TAG ; outputs under gpurun_out/TAG
#        CODE_ARGS="--code wimax_576_0.5 --snr 0.0 --frames 65536" tools/profile_tile.sh TAG  (config 2)
set -e
export LDPC_CN_SUB=0  # the split pass only re-derives the FETCH_SIZE factor on vn_kernel
TAG=${1:-prof_tile}
ARGS="${CODE_ARGS:-} --steps 2 --warmup 1 --cpu-seconds 0 --extra-snr= --point-snr= --phys-steps 0 --config4-snr= --config2 0 --config5 0 --dropin-calls 0"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_split -o run -- python3 bench.py ${CODE_ARGS:-} --split --schedule static --steps 1 --warmup 0 --iters 4 --cpu-seconds 0 --extra-snr= --point-snr= --phys-steps 0 --config4-snr= --config2 0 --config5 0 --dropin-calls 0 > $OUT/bench_fetch_split.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1
echo done
