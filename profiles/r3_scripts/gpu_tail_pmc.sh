#!/bin/bash
# PMC of the 3 dB streaming step (tail kernels): FETCH/WRITE and SQ counters, one --pmc pass each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tailpmc}; mkdir -p $O
ARGS="--snr 3.0 --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 0 --cpu-seconds 0 --extra-snr= --point-snr= --phys-steps 0 --dropin-calls 0"
run() { n=$1; shift; timeout -s KILL 300 rocprofv3 "$@" --output-format csv -d $O/$n -o run -- python3 bench.py $ARGS > $O/$n.log 2>&1 || { tail $O/$n.log; exit 1; }; echo "$n ok"; }
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE
run sq2 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS
python3 - $O <<'PY'
import csv, glob, sys, collections, json
o = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for n in ("fetch", "write", "sq1", "sq2"):
    for f in glob.glob(f"{o}/{n}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ldpc::(anonymous namespace)::", "").replace("ldpc::(anonymous namespace)::", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0))[:6]:
    t = tot[k]
    out = {c: t[c] for c in sorted(t)}
    if t.get("SQ_BUSY_CYCLES"):
        out["valu_busy_fraction"] = t["SQ_ACTIVE_INST_VALU"] / (t["SQ_BUSY_CYCLES"] * 4) if t["SQ_BUSY_CYCLES"] else None
    if t.get("SQ_WAVE_CYCLES"):
        out["wave_wait_fraction"] = t["SQ_WAIT_ANY"] / t["SQ_WAVE_CYCLES"]
        out["lds_busy_fraction"] = t.get("SQ_LDS_IDX_ACTIVE", 0) / max(t.get("SQ_BUSY_CYCLES", 1), 1)
    print(k, json.dumps({a: (round(b, 4) if isinstance(b, float) and b < 10 else b) for a, b in out.items()}))
PY
