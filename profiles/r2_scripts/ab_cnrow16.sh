#!/bin/bash
# cn_kernel vs the 16x40 cn_row_kernel shape (LDPC_CN_ROW16) on wimax_2304_0.5:
# the 3 dB streaming step (its tail runs on the split path) and the split path
# itself (static, 1 dB, 8,192 frames, T=10); two rounds.
set -o pipefail
O=gpurun_out/${TAG:-cnrow16}; mkdir -p $O
for round in 1 2; do
  for v in ${VS:-0 1}; do
    for cfg in t3 sp; do
      case $cfg in
        t3) A="--snr 3.0 --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 1";;
        sp) A="--split --schedule static --frames 8192 --iters 10 --steps 1 --warmup 1";;
      esac
      if [ "$v" = auto ]; then unset LDPC_CN_ROW16; else export LDPC_CN_ROW16=$v; fi
      timeout -k 10 200 python bench.py $A --cpu-seconds 0 --extra-snr= > $O/v${v}_${cfg}_$round.json 2> $O/v${v}_${cfg}_$round.err || { echo "FAIL $v $cfg"; exit 1; }
      python -c "
import json; d=json.loads(open('$O/v${v}_${cfg}_$round.json').read().strip().splitlines()[-1]); r=d['decode_roofline']
print('row16=$v $cfg r$round'.ljust(20), round(d['value']), 'cw/s', round(d['ms_per_step'],1), 'ms  cn', round(r['cn_ms'],1), 'vn', round(r['vn_ms'],1), d['fer'], d['avg_iters'])"
    done
  done
done
