set -o pipefail
O=gpurun_out/${TAG:-ab34}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_mc.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--steps 1 --warmup 1 --frames 16384 --cpu-seconds 0 --extra-snr="
timeout -k 10 200 python bench.py $B > $O/r12_new.json 2>/dev/null || exit 1
LDPC_HIP_LIB=variants/base.so timeout -k 10 200 python bench.py $B > $O/r12_base.json 2>/dev/null || exit 1
LDPC_TILE_SUB=1 timeout -k 10 200 python bench.py $B --code wimax_2304_0.75A > $O/r34_sub_new.json 2>/dev/null || exit 1
LDPC_TILE_SUB=1 LDPC_HIP_LIB=variants/base.so timeout -k 10 200 python bench.py $B --code wimax_2304_0.75A > $O/r34_sub_base.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py $B --code wimax_2304_0.75A > $O/r34_split.json 2>/dev/null || exit 1
for f in $O/*.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f',round(d['value']),r['kernel'],round(r['frac'],3),round(r['avg_launch_ms'],1),d['avg_iters'])"; done
