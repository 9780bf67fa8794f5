#!/bin/bash
# edge path tests + latency, and the physical key at 65,536 vs 262,144 frames per step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-edge3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_00_fork.py tests/test_gpu_edge.py tests/test_gpu_smallcols.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
BS=1,8,32 timeout -k 10 300 python -u tools/probe_small.py - > $O/lat.jsonl 2> $O/lat.err || { tail $O/lat.err; exit 1; }
cat $O/lat.jsonl
for pf in 65536 262144; do
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --frames 4096 --extra-snr= --point-snr= --cpu-seconds 0 --phys-frames $pf > $O/phys_$pf.json 2> $O/phys_$pf.err || { tail $O/phys_$pf.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/phys_$pf.json').read().strip().splitlines()[-1]);p=d['physical'];print($pf, round(p['value']), round(p['ms_per_step'],2), round(p['kernel_ms']/p['launches'],2), round(p['roofline']['frac'],3))"
done
