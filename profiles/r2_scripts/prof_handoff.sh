#!/bin/bash
# rocprofv3 kernel trace of one 3 dB streaming step with the hand-off (LDPC_HANDOFF=${HO:-1024})
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof_ho}; mkdir -p $O
LDPC_HANDOFF=${HO:-1024} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --snr 3.0 --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 0 --cpu-seconds 0 --extra-snr= > $O/bench.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, os
O=os.environ.get("TAG","prof_ho")
f=glob.glob(f"gpurun_out/{O}/trace/**/*kernel_trace.csv", recursive=True)[0]
rows=list(csv.DictReader(open(f)))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
t0=int(rows[0]["Start_Timestamp"])
agg={}
for r in rows:
    n=r["Kernel_Name"].split("(")[0][-40:]
    d=(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e6
    a=agg.setdefault(n,[0,0.0,1e9,0]); a[0]+=1; a[1]+=d; a[2]=min(a[2],d); a[3]=max(a[3],d)
for n,a in sorted(agg.items(), key=lambda x:-x[1][1]): print(f"{n:42s} n={a[0]:5d} total={a[1]:9.2f} ms min={a[2]:.3f} max={a[3]:.3f}")
last=max(int(r["End_Timestamp"]) for r in rows)
sub=[r for r in rows if "tile_sub_stream" in r["Kernel_Name"]]
for r in sub: print("sub-stream kernel: start", (int(r["Start_Timestamp"])-t0)/1e6, "end", (int(r["End_Timestamp"])-t0)/1e6, "ms")
print("last kernel end", (last-t0)/1e6, "ms")
PY
