#!/bin/bash
# wimax_576_0.5 across the BER-curve SNRs: tile-resident static schedule vs the
# streaming split schedule (GPU box)
mkdir -p gpurun_out/sched
for snr in 0.0 1.0 2.0 3.0; do
  for sch in static stream; do
    name=${sch}_${snr}
    timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --snr $snr --schedule $sch "$@" > gpurun_out/sched/$name.json 2> gpurun_out/sched/$name.err || { echo "FAIL $name"; tail -3 gpurun_out/sched/$name.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/sched/$name.json').read().strip().splitlines()[-1])
print('$name'.ljust(14), round(d['value']), 'cw/s', d['roofline']['kernel'], 'iters', round(d['avg_iters'],2), 'fer', round(d['fer'],4))"
  done
done
