#!/bin/bash
# BASELINE config 5 (DVB-S2 n=64800 r1/2 profile, physical mode, state in HBM:
# phys_cn_tile_kernel + phys_vn_tile_kernel) under rocprofv3 at each SNR given:
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in passes of their own
# (they cannot share a pass on gfx950).  8,192 frames, T = 50, the bench's
# config-5 frame source (`bench.py --mode physical --code dvbs2_profile_64800_0.5`).
# usage: tools/profile_config5.sh TAG [SNR ...]   (default: 1.0 -2.5)
# then:  python3 tools/summarize_config5.py gpurun_out/TAG profiles/TAG
set -o pipefail
TAG=${1:-prof_c5}; shift
SNRS=${*:-1.0 -2.5}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for X in $SNRS; do
    P="--mode physical --code dvbs2_profile_64800_0.5 --phys-hbm --snr $X --frames 8192 --steps 2 --warmup 1 --cpu-seconds 0 --extra-snr= --point-snr= --config4-snr= --dropin-calls 0"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$X -o run -- python3 bench.py $P > $OUT/trace_$X.log 2>&1 || exit 1
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$X -o run -- python3 bench.py $P > $OUT/fetch_$X.log 2>&1 || exit 1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$X -o run -- python3 bench.py $P > $OUT/write_$X.log 2>&1 || exit 1
done
echo done
