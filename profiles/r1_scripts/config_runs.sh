#!/bin/bash
# BASELINE.json configs 3 and 4 on one GPU (GPU box): bench.py lines into gpurun_out/configs/
mkdir -p gpurun_out/configs
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --steps 1 --warmup 0 --cpu-seconds 0 "$@" > gpurun_out/configs/$name.json 2> gpurun_out/configs/$name.err || { echo "FAIL $name"; tail -3 gpurun_out/configs/$name.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/configs/$name.json').read().strip().splitlines()[-1])
print('$name'.ljust(16), round(d['value']), 'cw/s', round(d['info_bits_per_s']/1e6,2), 'Mbit/s', d['config']['schedule'], d['roofline']['kernel'], 'iters', round(d['avg_iters'],2), 'fer', round(d['fer'],4), 'ber', '%.3g' % d['ber'])"
}
# config 3: wimax_2304_0.5, 50 iterations + early termination, batch 262,144 (16,384 resident)
for snr in 1.0 2.0 3.0; do run c3_${snr} --code wimax_2304_0.5 --frames 262144 --chunk 16384 --snr $snr; done
# config 4: wimax_2304_0.75A, sweep 1.0-4.0 dB, 32,768 frames per point (one GPU's shard of 262,144)
for snr in 1.0 1.5 2.0 2.5 3.0 3.5 4.0; do run c4_${snr} --code wimax_2304_0.75A --frames 32768 --chunk 16384 --snr $snr; done
