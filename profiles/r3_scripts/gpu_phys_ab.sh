#!/bin/bash
# physical-mode tests + the bench's physical key, old vs new library (two rounds)
set -o pipefail
O=gpurun_out/${TAG:-physab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_phys.py tests/test_phys_tile.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for round in 1 2; do for name in "$@"; do
  LDPC_HIP_LIB=variants/$name.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --frames 4096 --extra-snr= --point-snr= --cpu-seconds 0 > $O/${name}_$round.json 2> $O/${name}_$round.err || { tail $O/${name}_$round.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${name}_$round.json').read().strip().splitlines()[-1]);p=d['physical'];print('$name r$round', round(p['value']), round(p['ms_per_step'],2), round(p['kernel_ms']/p['launches'],2), round(p['roofline']['frac'],3), p['fer'], round(p['avg_iters'],4))"
done; done
