#!/bin/bash
# SQ counter passes of the tile-resident decoder (GPU box), one rocprofv3 run per pass.
# usage: tools/pmc_tile.sh TAG [bench args...]
TAG=${1:-pmc}; shift || true
ARGS=${@:---schedule static --frames 16384 --steps 1 --warmup 0 --cpu-seconds 0}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
pass() {
  local name=$1 ctrs=$2
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/$name -o run -- python3 bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -3 $OUT/$name.log; return 1; }
}
pass p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" &&
pass p2 "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" &&
pass p3 "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_IFETCH SQ_INST_CYCLES_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64"
echo done
