# Instruction-cache counters of the tile decoders, per library variant.
# usage (GPU box): TAG=x VARIANTS="a b" CODE=wimax_576_0.5 SNR=0.0 FRAMES=65536 bash tools/gpu_icache.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-icache}; mkdir -p $O
B="--code ${CODE:-wimax_576_0.5} --snr ${SNR:-0.0} --frames ${FRAMES:-65536} --steps 1 --warmup 0 --cpu-seconds 0 --extra-snr= --iters 10"
for v in $VARIANTS; do
  L=ldpc-simulator_amd/ldpc_amd/libldpc_hip.so; [ "$v" != new ] && L=variants/$v.so
  LDPC_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/$v -o run -- python3 bench.py $B > $O/$v.log 2>&1 || exit 1
done
echo done
