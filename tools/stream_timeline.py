#!/usr/bin/env python3
"""Host + device timeline of one me_search_pairs call from a rocprofv3 run with
--hip-trace --kernel-trace --memory-copy-trace (csv), e.g. of
tools/dbg/stream_trace.py.  Prints, for the last call, every HIP API call the
pipeline's thread made (start, host duration), every H2D copy and every search
kernel, in time order, in microseconds from the call's first upload; then the
per-batch summary: when each upload was enqueued and when it ran.
usage: python3 tools/stream_timeline.py <rocprof dir> [prefix=run]"""
import csv
import os
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    d = sys.argv[1]
    pre = sys.argv[2] if len(sys.argv) > 2 else "run"
    api = rows(os.path.join(d, f"{pre}_hip_api_trace.csv"))
    cp = rows(os.path.join(d, f"{pre}_memory_copy_trace.csv"))
    kr = rows(os.path.join(d, f"{pre}_kernel_trace.csv"))
    h2d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Correlation_Id"]))
                 for r in cp if r["Direction"].endswith("HOST_TO_DEVICE"))
    kern = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40],
                   int(r["Correlation_Id"])) for r in kr if "me_" in r["Kernel_Name"])
    # the last call: uploads after the largest gap between consecutive uploads
    gaps = [(h2d[i + 1][0] - h2d[i][1], i + 1) for i in range(len(h2d) - 1)]
    start_i = max(gaps)[1] if gaps else 0
    t0 = h2d[start_i][0]
    t1 = max(e for _, e, _, _ in kern)
    calls = [r for r in api if int(r["End_Timestamp"]) >= t0 - 2_000_000 and int(r["Start_Timestamp"]) <= t1]
    corr_api = {int(r["Correlation_Id"]): r for r in api}
    ev = []
    for r in calls:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ev.append((s, f"API  {r['Function']:<28} host {(e - s) / 1e3:8.1f} us  corr {r['Correlation_Id']}"))
    for s, e, c in h2d[start_i:]:
        a = corr_api.get(c)
        enq = (s - int(a["Start_Timestamp"])) / 1e3 if a else float("nan")
        ev.append((s, f"H2D  copy {(e - s) / 1e3:6.1f} us (ends {(e - t0) / 1e3:8.1f}); "
                      f"{enq:7.1f} us after its enqueue call began  corr {c}"))
    for s, e, n, c in kern:
        if e >= t0:
            ev.append((s, f"KERN {n} {(e - s) / 1e3:6.1f} us (ends {(e - t0) / 1e3:8.1f})  corr {c}"))
    for s, text in sorted(ev):
        if s >= t0 - 200_000:
            print(f"{(s - t0) / 1e3:9.1f}  {text}")


if __name__ == "__main__":
    main()
