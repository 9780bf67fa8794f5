#!/bin/bash
# Round evidence on one box after the test suite: the default bench line, the
# headline's rocprofv3 trace + PMC traffic (tools/profile_tile.sh), config 2's
# (the same script on wimax_576_0.5), config 4's sweep + static step
# (tools/profile_config4.sh) and config 5's two points (tools/profile_config5.sh).
# usage: TAG=r5z bash tools/gpu_profiles.sh   (outputs under gpurun_out/$TAG*)
# then:  tools/summarize_tile_profile.py gpurun_out/${TAG}_tile profiles/${TAG}_tile 663172 32768
#        tools/summarize_tile_profile.py gpurun_out/${TAG}_c2 profiles/${TAG}_c2 41278 65536
#        tools/summarize_config4.py gpurun_out/${TAG}_c4 profiles/${TAG}_c4
#        tools/summarize_config5.py gpurun_out/${TAG}_c5 profiles/${TAG}_c5
set -o pipefail
T=${TAG:-prof}
mkdir -p gpurun_out/$T
if [ -z "$NO_BENCH" ]; then
timeout -k 10 600 python -u bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { tail -30 gpurun_out/$T/bench_default.err; exit 1; }
python tools/bench_summary.py gpurun_out/$T/bench_default.json
fi
bash tools/profile_tile.sh ${T}_tile || exit 1
CODE_ARGS="--code wimax_576_0.5 --snr 0.0 --frames 65536" bash tools/profile_tile.sh ${T}_c2 || exit 1
bash tools/profile_config4.sh ${T}_c4 || exit 1
bash tools/profile_config5.sh ${T}_c5 || exit 1
echo profiles-done
