#!/bin/bash
# cn_long_kernel vs cn_kernel on wimax_2304_0.5 (GPU box): static chunk at 1 dB (50 iterations) and streaming at 3 dB.
set -o pipefail
mkdir -p gpurun_out/long
run() {
    local name=$1; shift
    env $ENVV timeout -k 10 300 python bench.py --cpu-seconds 0 --code wimax_2304_0.5 "$@" > gpurun_out/long/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/long/$name.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/long/$name.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name'.ljust(16), round(d['value']), 'cw/s  iters', round(d['avg_iters'],2), r['kernel'], round(r['avg_launch_ms'],3), 'ms x', r['launches'], ' frac', round(r['frac'],3), ' vn', round(d['decode_roofline']['vn_ms']/max(r['launches'],1),3))"
}
for v in "long:LDPC_CN_ROW=1" "old:LDPC_CN_ROW=0"; do
    tag=${v%%:*}; ENVV=${v#*:}
    run ${tag}_1dB --snr 1.0 --frames 16384 --steps 2 --warmup 1
    run ${tag}_3dB --snr 3.0 --frames 65536 --chunk 16384 --steps 2 --warmup 1
done
