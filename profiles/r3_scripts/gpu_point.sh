#!/bin/bash
# bench with the whole-point 3 dB entry (short headline), tail log on stderr.  TAG names gpurun_out/TAG.
set -o pipefail
O=gpurun_out/${TAG:-point}; mkdir -p $O
LDPC_TAIL_LOG=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-seconds 0 --phys-steps 0 ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
python -c "import json;d=json.load(open('$O/bench.json'));[print(p) for p in d['snr_points']]"
