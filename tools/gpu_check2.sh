set -o pipefail
O=gpurun_out/r2m; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ber_overlay.py -x -v -s --timeout 300 --timeout-method thread > $O/overlay.log 2>&1 || { echo OVERLAY_FAILED; tail -30 $O/overlay.log; }
grep -E "snr_db|passed|failed" $O/overlay.log | cut -c1-300
B="--steps 1 --warmup 1 --frames 16384 --cpu-seconds 0 --extra-snr= --code wimax_2304_0.75A"
timeout -k 10 200 python bench.py $B > $O/r34_split.json 2>/dev/null || exit 1
LDPC_TILE_SUB=1 timeout -k 10 200 python bench.py $B > $O/r34_sub.json 2>/dev/null || exit 1
for f in $O/*.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f',round(d['value']),r['kernel'],round(r['frac'],3),round(r['avg_launch_ms'],1),d['avg_iters'])"; done
