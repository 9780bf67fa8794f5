set -o pipefail
O=gpurun_out/${TAG:-st}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mc.py tests/test_gpu_tile.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|assert|FAIL" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--frames 16384 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr="
timeout -k 10 200 python bench.py $B --schedule static > $O/s1_static.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py $B --schedule stream > $O/s1_stream.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py $B --schedule stream --snr 3.0 --frames 65536 --chunk 16384 > $O/s3_stream.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py $B --schedule stream --snr 3.0 --frames 65536 --chunk 16384 --split > $O/s3_split.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py $B --schedule stream --snr 2.0 --frames 65536 --chunk 16384 > $O/s2_stream.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py $B --schedule stream --snr 2.0 --frames 65536 --chunk 16384 --split > $O/s2_split.json 2>/dev/null || exit 1
for f in $O/*.json; do python -c "import json,sys;d=json.load(open('$f'));r=d['roofline'];print('$f',round(d['value']),r['kernel'],round(r['frac'],3),round(r['avg_launch_ms'],1),round(d['avg_iters'],2),round(d['fer'],4))"; done
