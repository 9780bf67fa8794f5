#!/bin/bash
# Round-3 profile of one code's tile-resident decoder on the GPU box:
#   trace     rocprofv3 --kernel-trace --stats of bench.py (FRAMES, default 16,384; 1 dB, T=50)
#   fetch / write / fetch_split   FETCH_SIZE, WRITE_SIZE; FETCH_SIZE of the split
#             path's vn_kernel (reads every message once: the gfx950 FETCH_SIZE
#             correction factor, MI355X_MICROARCH.md HBM section)
#   sq1 / sq2 SQ counters (T=10), one --pmc pass each
# usage: CODE=... TAG=... tools/gpu_prof3.sh ; summarize with tools/summarize_prof3.py
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof3}; mkdir -p $O
C="--code ${CODE:-wimax_2304_0.5}"
B="$C --frames ${FRAMES:-16384} --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --phys-steps 0"
S="$C --frames 16384 --steps 1 --warmup 0 --iters 10 --cpu-seconds 0 --extra-snr= --phys-steps 0"
run() { n=$1; shift; timeout -s KILL 300 rocprofv3 "$@" --output-format csv -d $O/$n -o run -- python3 bench.py $ARGS > $O/$n.log 2>&1 || { tail $O/$n.log; exit 1; }; echo "$n ok"; }
ARGS=$B run trace --kernel-trace --stats
ARGS=$B run fetch --pmc FETCH_SIZE
ARGS=$B run write --pmc WRITE_SIZE
ARGS="$C --split --frames ${FRAMES:-16384} --steps 1 --warmup 0 --iters 4 --cpu-seconds 0 --extra-snr= --phys-steps 0" run fetch_split --pmc FETCH_SIZE
ARGS=$S run sq1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE
ARGS=$S run sq2 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS
echo done
