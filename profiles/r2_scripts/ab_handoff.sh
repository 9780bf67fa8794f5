#!/bin/bash
# Streaming tail: the sub-tile kernel alone (LDPC_HANDOFF=0) vs the hand-off to
# the column-parallel tail (default), bench's extra-SNR step shape (32,768
# frames through 8,192 slots) at 2 and 3 dB; two rounds.
set -o pipefail
O=gpurun_out/${TAG:-handoff}; mkdir -p $O
for round in 1 2; do
  for ho in ${HOS:-0 256 1024}; do
    for snr in 2.0 3.0; do
      if [ "$ho" = default ]; then unset LDPC_HANDOFF; else export LDPC_HANDOFF=$ho; fi
      timeout -k 10 200 python bench.py --snr $snr --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= > $O/ho${ho}_${snr}_$round.json 2> $O/ho${ho}_${snr}_$round.err || { echo "FAIL $ho $snr"; exit 1; }
      python -c "
import json; d=json.loads(open('$O/ho${ho}_${snr}_$round.json').read().strip().splitlines()[-1])
print('handoff=$ho snr=$snr r$round'.ljust(28), round(d['value']), 'cw/s', round(d['ms_per_step'],1), 'ms', d['fer'], d['avg_iters'])"
    done
  done
done
