#!/bin/bash
# Instruction-fetch counters of tile_kernel for each variants/*.so (GPU box):
# one rocprofv3 --pmc pass per library, 16,384 frames, one step.
export TMPDIR=/tmp
OUT=gpurun_out/icache
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -i -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST_ANY" $OUT/avail.txt | sort -u > $OUT/names.txt || true
cat $OUT/names.txt
for lib in variants/*.so; do
  name=$(basename $lib .so)
  export LDPC_HIP_LIB=$lib
  timeout -s KILL 120 rocprofv3 --pmc ${CTRS:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY} --output-format csv -d $OUT/$name -o run -- python3 bench.py --schedule static --frames 16384 --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
  python3 - $OUT/$name <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tile_kernel" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[1].split("/")[-1], dict(acc))
PY
done
