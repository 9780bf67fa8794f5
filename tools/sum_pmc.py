#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter CSVs per kernel: tools/sum_pmc.py DIR [kernel-substring]."""
import collections, csv, glob, sys
d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else ""
tot = collections.OrderedDict()
disp = collections.defaultdict(set)
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if ksub not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"][:60], r["Counter_Name"])
        tot[key] = tot.get(key, 0.0) + float(r["Counter_Value"])
        disp[key].add(r["Dispatch_Id"])
for (k, c), v in tot.items():
    print(f"{k:60s} {c:28s} {v:18.0f}  dispatches={len(disp[(k, c)])}")
