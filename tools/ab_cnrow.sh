#!/bin/bash
# A/B of the CN kernels on the headline workload (GPU box): env knobs of cn_row_kernel.
set -o pipefail
mkdir -p gpurun_out/cnrow
run() {  # name, env assignments...
    local name=$1; shift
    env "$@" timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/cnrow/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/cnrow/$name.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/cnrow/$name.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$name'.ljust(16), round(d['value']), 'cw/s  cn', round(r['avg_launch_ms'],3), 'ms  frac', round(r['frac'],3), ' vn', round(d['decode_roofline']['vn_ms']/r['launches'],3))"
}
for cfg in "w8 LDPC_CN_ROW=8" "w8_g2048 LDPC_CN_ROW=8 LDPC_CN_ROW_GRID=2048" "w8_g4096 LDPC_CN_ROW=8 LDPC_CN_ROW_GRID=4096" \
           "w16 LDPC_CN_ROW=16" "w16_g1024 LDPC_CN_ROW=16 LDPC_CN_ROW_GRID=1024" "w4 LDPC_CN_ROW=4" "old LDPC_CN_ROW=0"; do
    run $cfg
done
