#!/usr/bin/env python3
"""Fold rocprofv3 outputs of tools/profile.sh into profiles/.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
are in KiB (x1024); on gfx950 FETCH_SIZE reports exactly half the bytes of a
wide coalesced (16 B/lane) streaming read, so it is doubled; WRITE_SIZE is
exact for such stores.  The counters come from separate passes.

bench.py launches a kernel at more than one size in one run (the timed F-frame
batch, then F one-frame parity calls on the same persistent grid), so every
per-launch figure (time, FETCH, WRITE) is taken over the kernel's *batch*
launches only: dispatches lasting at least half the kernel's longest one in
that pass.  The one-frame launches are reported beside them ("single").
"""
import csv
import glob
import json
import os
import shutil
import sys

out_dir, tag = sys.argv[1], sys.argv[2]
args = sys.argv[3:]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")
os.makedirs(PROF, exist_ok=True)


def rows(pattern):
    files = glob.glob(os.path.join(out_dir, "**", pattern), recursive=True)
    out = []
    for f in files:
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out, files


stats, sfiles = rows("*kernel_stats.csv")
for f in sfiles:
    shutil.copy(f, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
ktrace, _ = rows("*kernel_trace.csv")


def is_me(name):
    return "me_" in name or "qsad" in name or "generic" in name


def split(per):
    """{kernel: [(duration_ns, value)]} -> {kernel: (batch mean, single mean or None, n batch)}"""
    out = {}
    for k, v in per.items():
        top = max(d for d, _ in v)
        big = [x for d, x in v if d >= 0.5 * top]
        small = [x for d, x in v if d < 0.5 * top]
        out[k] = (sum(big) / len(big), sum(small) / len(small) if small else None, len(big))
    return out


def counter(pattern, cname):
    rs, _ = rows(pattern)
    per = {}
    for r in rs:
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if r.get("Counter_Name") != cname or not is_me(name):
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per.setdefault(name, []).append((dur, float(r["Counter_Value"])))
    return split(per)


def trace_times():
    per = {}
    for r in ktrace:
        name = r.get("Kernel_Name", "")
        if is_me(name):
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per.setdefault(name, []).append((dur, float(dur)))
    return split(per)


fetch = counter("*counter_collection.csv", "FETCH_SIZE")
write = counter("*counter_collection.csv", "WRITE_SIZE")
times = trace_times()
# optional passes (profile.sh SIZED=1): read requests by size, L2 hits / misses
sized = {c: counter("*counter_collection.csv", c) for c in
         ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum",
          "TCC_EA0_RDREQ_sum", "TCC_HIT_sum", "TCC_MISS_sum",
          # profile.sh VALU=1: instruction counts (wave-level, all SQs)
          "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_WAVES")}
summary = {}
for r in stats:
    name = r.get("Name", "")
    if not is_me(name):
        continue
    summary[name] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                     "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
for name, (big, small, n) in times.items():
    e = summary.setdefault(name, {})
    e.update({"batch_calls": n, "batch_avg_ns": big, "single_avg_ns": small})
for name, (big, small, _) in fetch.items():
    summary.setdefault(name, {}).update({"fetch_kib": big, "single_fetch_kib": small})
for name, (big, small, _) in write.items():
    summary.setdefault(name, {}).update({"write_kib": big, "single_write_kib": small})
dom = max(summary, key=lambda k: summary[k].get("avg_ns", 0) * summary[k].get("calls", 0))
d = summary[dom]
for c, per in sized.items():
    for name, (big, small, _) in per.items():
        summary.setdefault(name, {}).update({c: big, "single_" + c: small})
hbm = hbm_single = None
if "fetch_kib" in d and "write_kib" in d:
    hbm = 2 * d["fetch_kib"] * 1024 + d["write_kib"] * 1024
    if d.get("single_fetch_kib") is not None and d.get("single_write_kib") is not None:
        hbm_single = 2 * d["single_fetch_kib"] * 1024 + d["single_write_kib"] * 1024
# read bytes from the request sizes, where that pass ran
rd_sized = None
if all(k in d for k in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
    rd_sized = (32 * d["TCC_EA0_RDREQ_32B_sum"] + 64 * d["TCC_EA0_RDREQ_64B_sum"] +
                128 * d["TCC_EA0_RDREQ_128B_sum"])
# every kernel of one search (the SSD prepass beside its main kernel): bytes per
# launch of each, weighted by its launches per dominant-kernel launch
search = 0.0
for k, v in summary.items():
    if "fetch_kib" in v and "write_kib" in v and v.get("calls"):
        per = v.get("batch_calls", v["calls"]) / max(d.get("batch_calls", d.get("calls", 1)), 1)
        search += per * (2 * v["fetch_kib"] * 1024 + v["write_kib"] * 1024)
bench_tag = None
cfg = "1080p"
cost = "sad"
frames = 16  # bench.py --frames-per-step default
for i, a in enumerate(args):
    if a == "--config":
        cfg = args[i + 1]
    if a == "--cost":
        cost = args[i + 1]
    if a == "--frames-per-step":
        frames = int(args[i + 1])
blk, span = {"1080p": (16, 32), "4k": (16, 64), "8k": (8, 128)}[cfg]
# keyed like bench.py's lookup: the workload and its frames per step (a SAD
# launch holds every frame of the step, an SSD launch one frame)
bench_tag = f"{cfg}_b{blk}_s{span}_{cost}_f{frames}"
if os.environ.get("ME_PATH") == "lean":  # the lean matrix-core SSD path (S2 in the search kernel)
    bench_tag += "_lean"
bench_tag += os.environ.get("PMC_KEY_SUFFIX", "")  # A/B variants (tuning-build settings)
path = os.path.join(PROF, "pmc_summary.json")
try:
    allsum = json.load(open(path))
except (OSError, ValueError):
    allsum = {}
allsum[bench_tag] = {"profile_tag": tag, "dominant_kernel": dom, "kernels": summary,
                     "hbm_bytes_per_launch": hbm,
                     "hbm_bytes_per_single_frame_launch": hbm_single,
                     "read_bytes_by_request_size": rd_sized,
                     "hbm_bytes_per_search": search or None,
                     "note": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 correction, "
                             "MI355X_MICROARCH.md §HBM); separate --pmc passes; per_launch: the "
                             "dominant kernel's batch launches (>= half its longest); "
                             "per_search: every kernel of one search"}
json.dump(allsum, open(path, "w"), indent=1)
print(json.dumps(allsum[bench_tag], indent=1))
