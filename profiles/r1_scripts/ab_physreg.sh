#!/bin/bash
# A/B of the LDS physical kernels (GPU box): phys_kernel vs phys_reg_kernel at 4 / 6 waves per SIMD.
set -o pipefail
mkdir -p gpurun_out/physreg
run() {  # name, bench args..., env via ENVV
    local name=$1; shift
    env $ENVV timeout -k 10 300 python bench.py --mode physical --cpu-seconds 0 --steps 3 --warmup 1 "$@" > gpurun_out/physreg/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/physreg/$name.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/physreg/$name.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name'.ljust(22), round(d['value']), 'cw/s  iters', round(d['avg_iters'],2), ' fer', round(d['fer'],4), ' phys', round(r['avg_launch_ms'],3), 'ms')"
}
for v in "reg:LDPC_PHYS_REG=1"; do
    tag=${v%%:*}; ENVV=${v#*:}
    run ${tag}_2304h_0 --code wimax_2304_0.5 --snr 0.0
    run ${tag}_2304h_-2.5 --code wimax_2304_0.5 --snr -2.5
    run ${tag}_2304A_0 --code wimax_2304_0.75A --snr 0.0
    run ${tag}_576_0 --code wimax_576_0.5 --snr 0.0
    run ${tag}_576_-2.5 --code wimax_576_0.5 --snr -2.5
done
