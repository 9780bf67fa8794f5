#!/bin/bash
# Counter breakdown of the headline kernel (tile_sub_kernel<4>, config 3:
# wimax_2304_0.5, 1 dB, T = 50) -- where its time and its extra reads go.
# One rocprofv3 --pmc pass per counter group (each within the gfx950 per-block
# slot limits: <= 4 TCC, <= 8 SQ, <= 4 TCP), every pass under its own timeout.
#   l2      TCC_HIT / TCC_MISS (L2 hit rate of every request)
#   ea      TCC_EA0_RDREQ / _32B / TCC_EA0_RDREQ_DRAM (fabric reads, DRAM reads)
#   ea_w    TCC_EA0_WRREQ / _64B
#   tcp     L1 (vector cache) requests and misses to L2
#   sqwait  wave-cycles issuing / parked / issue-stalled
#   sqinst  instruction mix per wavefront
# Then the same L2 pass at 2,048 frames (128 workgroups, 16 per XCD: half the
# posterior working set per L2) beside 4,096 (256 workgroups, one per CU).
# usage: tools/profile_counters.sh TAG [FRAMES] [ITERS]; outputs under gpurun_out/TAG
#   PASSES="sqwait sqinst" runs only those passes; CODE_ARGS="--code wimax_2304_0.75A" another code
set -o pipefail
TAG=${1:-counters}
FR=${2:-32768}
IT=${3:-50}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="${CODE_ARGS:-} --frames $FR --iters $IT --steps 1 --warmup 0 --cpu-seconds 0 --extra-snr= --point-snr= --phys-steps 0 --config4-snr= --config2 0 --config5 0 --dropin-calls 0"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
pass() {  # name, counters...
  local name=$1; shift
  if [ -n "$PASSES" ] && ! echo " $PASSES " | grep -q " $name "; then return 0; fi
  echo "pass $name: $*"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed ($?)"; tail -5 $OUT/$name.log; return 1; }
}
pass l2 TCC_HIT_sum TCC_MISS_sum || exit 1
pass ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum || exit 1
pass ea_w TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum || exit 1
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum || exit 1
pass sqwait SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS || exit 1
pass sqinst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH || exit 1
[ -n "$PASSES" ] && { echo counters-done; exit 0; }
for fr in 2048 4096; do
  A2="--frames $fr --iters $IT --steps 1 --warmup 0 --cpu-seconds 0 --extra-snr= --point-snr= --phys-steps 0 --config4-snr= --config2 0 --config5 0 --dropin-calls 0"
  echo "pass l2_$fr"
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/l2_$fr -o run -- python3 bench.py $A2 > $OUT/l2_$fr.log 2>&1 || { echo "pass l2_$fr failed"; exit 1; }
done
echo counters-done
