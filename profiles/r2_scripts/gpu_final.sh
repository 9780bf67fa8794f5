set -o pipefail
O=gpurun_out/${TAG:-final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err && python -c "import json;d=json.load(open('$O/bench_default.json'));print(round(d['value']),d['roofline']['kernel'],round(d['roofline']['frac'],3),[ (p['snr_db'],round(p['value'])) for p in d.get('snr_points',[])])"
bash tools/profile_tile.sh ${TAG:-final}_prof && echo PROF_OK
