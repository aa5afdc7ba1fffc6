#!/usr/bin/env python3
"""Average rocprofv3 counter values per kernel from a counter_collection.csv tree.
usage: pmc_counters.py <dir> [kernel-substring]"""
import csv, glob, os, sys
d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "me_"
acc = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if sub not in name:
            continue
        key = (name.split("(")[0][:60], r["Counter_Name"])
        acc.setdefault(key, []).append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:60s} {c:28s} n={len(v):3d} avg={sum(v)/len(v):.6g}")
