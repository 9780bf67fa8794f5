#!/bin/bash
# tile8 diagnostics: phase timers (diag build) + SQ counters, tile8 vs tile_sub (LDPC_TILE8=0).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-t8b}; mkdir -p $O
B="--frames 4096 --steps 1 --warmup 0 --cpu-seconds 0 --extra-snr= --phys-steps 0"
LDPC_HIP_LIB=variants/t8diag.so timeout -k 10 200 python -u bench.py $B > $O/timers.log 2>&1 || { tail -20 $O/timers.log; exit 1; }
grep "^T8" $O/timers.log | head -40
P="--steps 1 --warmup 0 --frames 16384 --cpu-seconds 0 --extra-snr= --phys-steps 0 --iters 10"
for v in new old; do
  E=""; [ $v = old ] && E="LDPC_TILE8=0"
  env $E timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/${v}_p1 -o run -- python3 bench.py $P > $O/${v}_p1.log 2>&1 || exit 1
  env $E timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --output-format csv -d $O/${v}_p2 -o run -- python3 bench.py $P > $O/${v}_p2.log 2>&1 || exit 1
  env $E timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${v}_p3 -o run -- python3 bench.py $P > $O/${v}_p3.log 2>&1 || exit 1
  python3 tools/sum_pmc.py $O/${v}_p1 tile; python3 tools/sum_pmc.py $O/${v}_p2 tile; python3 tools/sum_pmc.py $O/${v}_p3 tile
done
