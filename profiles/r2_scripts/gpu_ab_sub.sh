set -o pipefail
O=gpurun_out/${TAG:-ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tile.py -x -q --timeout 200 --timeout-method thread > $O/tile_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tile_tests.log; exit 1; }
tail -1 $O/tile_tests.log
B="--steps 1 --warmup 1 --frames 16384 --cpu-seconds 0 --extra-snr="
for round in 1 2; do
  timeout -k 10 200 python bench.py $B > $O/new_$round.json 2>/dev/null || exit 1
  for v in $VARIANTS; do LDPC_HIP_LIB=variants/$v.so timeout -k 10 200 python bench.py $B > $O/${v}_$round.json 2>/dev/null || exit 1; done
done
for f in $O/*.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f',round(d['value']),r['kernel'],round(r['frac'],3),round(r['avg_launch_ms'],1),d['avg_iters'])"; done
