#!/usr/bin/env python3
"""Fold tools/dbg/pmc_variants.sh passes: per variant, the dominant kernel's
batch launches (>= half its longest) -> mean read bytes from request sizes,
L2 hit rate and mean duration under counters."""
import csv
import glob
import os
import sys

out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "v*/")), key=lambda p: int(p.rstrip("/").split("v")[-1])):
    name = open(d.rstrip("/") + ".variant").read().strip()
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "me_" in r["Kernel_Name"]]
    per = {}
    for r in rows:
        k = (r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])
        e = per.setdefault(k, {"dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    if not per:
        print(f"{name:40s} no kernels")
        continue
    kern = max({k for k, _ in per}, key=lambda n: sum(v["dur"] for (kk, _), v in per.items() if kk == n))
    ds = [v for (k, _), v in per.items() if k == kern]
    top = max(v["dur"] for v in ds)
    big = [v for v in ds if v["dur"] >= 0.5 * top]
    mean = lambda key: sum(v.get(key, 0) for v in big) / len(big)
    if "TCC_EA0_RDREQ_128B_sum" in big[0]:
        rd = 128 * mean("TCC_EA0_RDREQ_128B_sum") + 64 * mean("TCC_EA0_RDREQ_64B_sum")
        h, m = mean("TCC_HIT_sum"), mean("TCC_MISS_sum")
        print(f"{name:40s} {kern[-40:]:40s} n {len(big):3d}  {mean('dur') / 1e3:9.1f} us  "
              f"read {rd / 1e6:8.1f} MB  L2 hit {h / max(h + m, 1):.4f}")
    else:  # any other counter set: every counter's batch-launch mean
        cs = sorted(k for k in big[0] if k != "dur")
        print(f"{name:40s} {kern[-40:]:40s} n {len(big):3d}  {mean('dur') / 1e3:9.1f} us  " +
              "  ".join(f"{c} {mean(c):.4g}" for c in cs))
