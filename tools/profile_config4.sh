#!/bin/bash
# BASELINE config 4 under rocprofv3 (tools/config4_run.py: the bench's config4
# sweep, then its static 1 dB step, each alone in its process): kernel trace +
# stats, then one PMC pass per TCC counter (FETCH_SIZE and WRITE_SIZE cannot
# share a pass on gfx950).  Outputs under gpurun_out/$TAG.
# then: python3 tools/summarize_config4.py gpurun_out/TAG profiles/TAG
set -o pipefail
TAG=${1:-prof_c4}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for M in sweep static; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${M}_trace -o run -- python3 tools/config4_run.py $M > $OUT/${M}_trace.log 2>&1 || exit 1
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${M}_fetch -o run -- python3 tools/config4_run.py $M > $OUT/${M}_fetch.log 2>&1 || exit 1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${M}_write -o run -- python3 tools/config4_run.py $M > $OUT/${M}_write.log 2>&1 || exit 1
done
echo done
