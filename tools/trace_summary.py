#!/usr/bin/env python3
"""Per-launch duration summary of a rocprofv3 --kernel-trace run, per kernel:
launch count, mean, median, p10, p90, min, max (ns).  The committed
`*_kernel_stats.csv` averages every launch of a kernel, the timed batched
launches and the one-frame parity re-searches alike; this keeps them apart.
usage: python3 tools/trace_summary.py <profile dir> <label> > profiles/<tag>_kernel_trace_summary.txt"""
import csv
import glob
import os
import sys


def main():
    d, label = sys.argv[1], sys.argv[2]
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "me_" not in name:
                continue
            short = name.split("(")[0].split("<")[0].split()[-1].split("::")[-1]
            per.setdefault(short, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"# per-launch durations (ns) from rocprofv3 --kernel-trace of {label}; "
          "bench.py's timed launches are the long ones")
    def line(k, tag, v):
        v = sorted(v)
        n = len(v)
        q = lambda p: v[min(n - 1, int(p * n))]
        print(f"{k}{tag}: launches {n}, mean {sum(v) / n:.0f}, median {q(0.5)}, p10 {q(0.1)}, "
              f"p90 {q(0.9)}, min {v[0]}, max {v[-1]}")

    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        line(k, "", v)
        # batched launches (>= half the longest, as tools/pmc_summary.py splits
        # them) apart from the short one-frame parity re-searches
        big = [x for x in v if x >= max(v) / 2]
        small = [x for x in v if x < max(v) / 2]
        if small and big:
            line(k, " [batched, >= max/2]", big)
            line(k, " [short, < max/2]", small)


if __name__ == "__main__":
    main()
