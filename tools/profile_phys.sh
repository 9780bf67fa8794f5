#!/bin/bash
# Physical mode: rocprofv3 trace + VALU counters of
# phys_reg_kernel (its state lives in LDS: the bound is VALU issue, not HBM),
# then the split streaming path's drain tail at 3 dB (config 3, SURVEY §8 d).
# usage: tools/profile_phys.sh TAG ; outputs under gpurun_out/TAG
set -e
TAG=${1:-prof_phys}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
P="--mode physical --snr 0.0 --frames 65536 --steps 2 --warmup 1 --cpu-seconds 0 --extra-snr="
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/phys_trace -o run -- python3 bench.py $P > $OUT/phys_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/phys_sq -o run -- python3 bench.py $P > $OUT/phys_sq.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/phys_grbm -o run -- python3 bench.py $P > $OUT/phys_grbm.log 2>&1
S="--snr 3.0 --frames 32768 --chunk 16384 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --schedule stream"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tail_trace -o run -- python3 bench.py $S > $OUT/tail_trace.log 2>&1
python3 bench.py $S > $OUT/tail_bench.json 2>/dev/null
echo done
