#!/bin/bash
# Streaming vs static Monte-Carlo schedule, same frames (GPU box).
set -o pipefail
mkdir -p gpurun_out/stream
run() {  # name, args...
    local name=$1; shift
    timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" > gpurun_out/stream/$name.log 2>&1 || { echo "FAILED $name"; cat gpurun_out/stream/$name.log | tail -5; exit 1; }
    python - "$name" gpurun_out/stream/$name.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s} {d['value']:12.1f} cw/s  avg_iters {d['avg_iters']:.2f}  fer {d['fer']:.4f}  cn {d['roofline']['avg_launch_ms']:.3f} ms x{d['roofline']['launches']}  frac {d['roofline']['frac']:.3f}")
PY
}
for sched in stream static; do
    run 576_0dB_$sched --schedule $sched --steps 3 --warmup 1
done
for code in wimax_2304_0.5 wimax_2304_0.75A; do
  for snr in 1.0 3.0; do
    for sched in stream static; do
        run ${code}_${snr}_$sched --code $code --snr $snr --frames 65536 --chunk 16384 --schedule $sched --steps 2 --warmup 1
    done
  done
done
