set -o pipefail
O=gpurun_out/r2k; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --mode physical --snr 0.0 --frames 65536 --steps 2 --warmup 1 --extra-snr= > $O/bench_phys.json 2> $O/bench_phys.err && cut -c1-200 $O/bench_phys.json
timeout -k 10 300 python -u bench.py --code wimax_576_0.5 --snr 0.0 --frames 65536 --extra-snr= --cpu-seconds 0 > $O/bench_576.json 2> $O/bench_576.err && cut -c1-300 $O/bench_576.json
