#!/usr/bin/env python3
"""Search-kernel start delays of a pair-pipeline trace (rocprofv3 --hip-trace
--kernel-trace --memory-copy-trace, csv; tools/dbg/stream_trace.sh): for every
search launch, how long after (a) the previous search ended, (b) its launch
call returned on the host and (c) the last of the five uploads enqueued
before it landed did it start.  The gate is the latest of the three.
usage: python3 tools/stream_gaps.py <rocprof dir>"""
import csv,sys
d=sys.argv[1]
api=list(csv.DictReader(open(d+'/run_hip_api_trace.csv')))
cp=list(csv.DictReader(open(d+'/run_memory_copy_trace.csv')))
kr=[r for r in csv.DictReader(open(d+'/run_kernel_trace.csv')) if 'me_' in r['Kernel_Name']]
byc={int(r['Correlation_Id']):r for r in api}
h2d=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp']),int(r['Correlation_Id'])) for r in cp if 'HOST_TO' in r['Direction'])
ks=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp']),int(r['Correlation_Id'])) for r in kr)
prev_end=None
for s,e,c in ks:
    a=byc.get(c)
    launch_end=int(a['End_Timestamp']) if a else 0
    # uploads enqueued before this launch call (corr < c) and after previous kernel's corr
    ups=[x for x in h2d if x[2]<c]
    last_up=max(x[1] for x in ups[-5:]) if ups else 0
    cands={'prev_kernel_end':prev_end or 0,'launch_call_end':launch_end,'last5_upload_end':last_up}
    gate=max(cands.values())
    print(f"kern {c}: start-gate {(s-gate)/1e3:7.1f} us; prev_end {((s-(prev_end or s))/1e3):7.1f} launch {((s-launch_end)/1e3):7.1f} upl {((s-last_up)/1e3):7.1f}  dur {(e-s)/1e3:.1f}")
    prev_end=e
