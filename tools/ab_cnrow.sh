#!/bin/bash
# A/B of the CN kernels on the headline workload (GPU box): env knobs of cn_row_kernel.
set -o pipefail
mkdir -p gpurun_out/cnrow
run() {  # name, env assignments...
    local name=$1; shift
    env LDPC_AB=1 "$@" timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/cnrow/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/cnrow/$name.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/cnrow/$name.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name'.ljust(16), round(d['value']), 'cw/s  cn', round(r['avg_launch_ms'],3), 'ms  frac', round(r['frac'],3), ' vn', round(d['decode_roofline']['vn_ms']/r['launches'],3))"
}
for cfg in "v0_s3w6 LDPC_CN_ROW_VARIANT=0" "v2_s4w6 LDPC_CN_ROW_VARIANT=2" "v3_s4w8 LDPC_CN_ROW_VARIANT=3" "v4_s6w8 LDPC_CN_ROW_VARIANT=4" "v5_s3w8 LDPC_CN_ROW_VARIANT=5" "v1_s1w4 LDPC_CN_ROW_VARIANT=1"; do
    run $cfg
done
