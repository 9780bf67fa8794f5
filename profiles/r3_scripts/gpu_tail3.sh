#!/bin/bash
# kernel trace of bench's 3 dB streaming step (32,768 frames through 8,192 slots)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tail3}; mkdir -p $O
S="--snr 3.0 --schedule stream --chunk 8192 --frames 32768 --steps 1 --warmup 1 --cpu-seconds 0 --extra-snr= --point-snr= --phys-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $S > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/'+__import__('os').environ.get('TAG','tail3')+'/trace/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]: print(r['Name'][:50], r['Calls'], round(float(r['TotalDurationNs'])/1e6,1), 'ms')
f=glob.glob('gpurun_out/'+__import__('os').environ.get('TAG','tail3')+'/trace/**/*kernel_trace.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
t0=min(int(r['Start_Timestamp']) for r in rows)
cn=[r for r in rows if 'cn_kernel' in r['Kernel_Name']]
print('cn launches', len(cn))
for r in cn[::4]: print(round((int(r['Start_Timestamp'])-t0)/1e6,1), round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6,2), r.get('Grid_Size_X', r.get('Grid_Size','')))
PY
