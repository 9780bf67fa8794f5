#!/bin/bash
# Physical mode: config 5 (DVB-S2-profile, HBM tiles) and LDS vs HBM on WiMAX 2304 (GPU box).
set -o pipefail
mkdir -p gpurun_out/phys
run() {  # name, args...
    local name=$1; shift
    timeout -k 10 300 python bench.py "$@" > gpurun_out/phys/$name.log 2>&1 || { echo "FAILED $name"; tail -5 gpurun_out/phys/$name.log; exit 1; }
    python - "$name" gpurun_out/phys/$name.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]; cb = d.get("cpu_baseline") or {}
print(f"{sys.argv[1]:28s} {d['value']:12.1f} cw/s  avg_iters {d['avg_iters']:.2f}  fer {d['fer']:.4f}  "
      f"{r['kernel']} {r['avg_launch_ms']:.3f} ms x{r['launches']}  frac {r.get('frac', float('nan')):.3f}  cpu {cb.get('value', 0):.1f}")
PY
}
run dvbs2_1.0 --mode physical --code dvbs2_profile_64800_0.5 --snr 1.0 --frames 1024 --steps 5 --warmup 1 --cpu-seconds 10
run dvbs2_-2.5 --mode physical --code dvbs2_profile_64800_0.5 --snr -2.5 --frames 1024 --steps 3 --warmup 1 --cpu-seconds 0
run dvbs2_1.0_8k --mode physical --code dvbs2_profile_64800_0.5 --snr 1.0 --frames 8192 --steps 3 --warmup 1 --cpu-seconds 0
run w2304_lds_0.0 --mode physical --code wimax_2304_0.5 --snr 0.0 --frames 65536 --steps 3 --warmup 1 --cpu-seconds 0
run w2304_hbm_0.0 --mode physical --phys-hbm --code wimax_2304_0.5 --snr 0.0 --frames 65536 --chunk 16384 --steps 3 --warmup 1 --cpu-seconds 0
run w576_hbm_-2.5 --mode physical --phys-hbm --code wimax_576_0.5 --snr -2.5 --frames 65536 --steps 3 --warmup 1 --cpu-seconds 0
run w576_lds_-2.5 --mode physical --code wimax_576_0.5 --snr -2.5 --frames 65536 --steps 3 --warmup 1 --cpu-seconds 0
