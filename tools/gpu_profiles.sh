#!/bin/bash
# Round evidence on one box after the test suite: the default bench line, the
# headline's rocprofv3 trace + PMC traffic (tools/profile_tile.sh), the
# physical mode's VALU counts at its two SNR points (tools/profile_phys.sh) and
# config 4's sweep + static step (tools/profile_config4.sh).
# usage: TAG=r4p bash tools/gpu_profiles.sh   (outputs under gpurun_out/$TAG*)
set -o pipefail
T=${TAG:-prof}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { tail -30 gpurun_out/$T/bench_default.err; exit 1; }
python tools/bench_summary.py gpurun_out/$T/bench_default.json
bash tools/profile_tile.sh ${T}_tile || exit 1
bash tools/profile_phys.sh ${T}_phys 1.0 -2.5 || exit 1
bash tools/profile_config4.sh ${T}_c4 || exit 1
echo profiles-done
