"""Sum one PMC counter per kernel name over a rocprofv3 --pmc output dir:
   python tools/dbg/pmc_kernel_sum.py <dir> <COUNTER>  -> name: calls, mean value"""
import csv, glob, sys, os
d, c = sys.argv[1], sys.argv[2]
per = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r.get("Counter_Name") != c:
            continue
        n = (r.get("Kernel_Name") or "").split("(")[0].split("<")[0].split()[-1] if r.get("Kernel_Name") else "?"
        per.setdefault(n, []).append(float(r["Counter_Value"]))
for n, v in sorted(per.items()):
    if "me_" in n:
        print(f"{c} {n}: calls {len(v)} mean {sum(v)/len(v):.1f}")
