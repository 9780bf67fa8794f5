#!/bin/bash
# Physical mode: per SNR point, a rocprofv3 kernel trace and
# one PMC pass of SQ counters over `bench.py --mode physical` -- the VALU
# instructions per frame-iteration of phys_reg_kernel (its state lives in LDS:
# the bound is VALU issue, not HBM) that bench.py's physical roofline prices
# against (committed_valu: code, kernel and SNR must match).
# usage: tools/profile_phys.sh TAG [SNR ...]   (default SNRs: 1.0 -2.5)
# then:  python3 tools/summarize_phys_profile.py gpurun_out/TAG profiles/TAG
set -o pipefail
TAG=${1:-prof_phys}; shift
SNRS=${*:-1.0 -2.5}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for X in $SNRS; do
    P="--mode physical --snr $X --frames 262144 --steps 2 --warmup 1 --cpu-seconds 0 --extra-snr= --point-snr= --config4-snr= --dropin-calls 0"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$X -o run -- python3 bench.py $P > $OUT/trace_$X.log 2>&1 || exit 1
    timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq_$X -o run -- python3 bench.py $P > $OUT/sq_$X.log 2>&1 || exit 1
done
echo done
