#!/usr/bin/env python3
"""Per-wave timeline of the SAD flow kernel from the ME_STAMPS diagnostic build
(libme_hip_stamps.so): start-up delay to the first task, time spent waiting for
items, tasks per wave, and how the waves / CUs finish.  Diagnostic only (the
stamps cost cycles themselves); times in shader cycles unless marked.
usage: python3 tools/flow_stamps.py [r0:r1 (one stripe's block rows: the split mode)]"""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from motionestimation_amd import _lib, synth
_lib.LIB_PATH = os.path.join(REPO, "motionestimation_amd", "lib", "libme_hip_stamps.so")
import ctypes
import motionestimation_amd as me

ref, cur = synth.named_pair("1080p")
eng = me.Engine(devices=[0])
rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
n = me.num_blocks(1920, 1080, 16)
mv = torch.empty((n, 2), dtype=torch.int16, device="cuda")
co = torch.empty(n, dtype=torch.int32, device="cuda")
rows = sys.argv[1] if len(sys.argv) > 1 else ""
if rows.startswith("batch"):  # batchF: F frames in one launch (me_full_search_batch_device)
    F = int(rows[5:])
    rows = ""
    rb = torch.from_numpy(np.stack([ref] * F)).cuda()
    cb = torch.from_numpy(np.stack([cur] * F)).cuda()
    mvb = torch.empty((F * n, 2), dtype=torch.int16, device="cuda")
    cob = torch.empty(F * n, dtype=torch.int32, device="cuda")
    for _ in range(40):  # past the clock ramp (tools/dbg/ramp_probe.py)
        eng.search_batch_device(rb, 0, cb, 0, 1920, 1080, 16, 32, "sad", 0, 68, mvb, cob)
else:
    for _ in range(400):  # past the clock ramp (tools/dbg/ramp_probe.py)
        eng.full_search_device(rt, ct, 16, 32, "sad", mv, co)
for _ in range(20):
    if "F" in dir() and not rows:
        eng.search_batch_device(rb, 0, cb, 0, 1920, 1080, 16, 32, "sad", 0, 68, mvb, cob)
    elif rows:
        a, b = (int(x) for x in rows.split(":"))
        eng.search_stripe_device(rt, 0, ct, 0, 1920, 1080, 16, 32, "sad", a, b, mv, co)
    else:
        eng.full_search_device(rt, ct, 16, 32, "sad", mv, co)
torch.cuda.synchronize()
L = _lib.lib()
L.me_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(8 << 16, np.uint64)
L.me_debug_stamps(buf.ctypes.data, buf.size)
st = buf.reshape(-1, 8)[:4096].astype(np.int64)
if os.environ.get("FLOW_STAMPS_SAVE"):  # raw per-wave records for offline analysis
    np.save(os.environ["FLOW_STAMPS_SAVE"], st)
st = st[st[:, 0] > 0]
start, first, end, spin, ntask = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4]
r0, r1 = st[:, 5], st[:, 6]
life = end - start
print(f"waves {len(st)}; tasks per wave: {np.bincount(ntask)}")
print(f"start -> first task (cycles): median {np.median(first - start):.0f} p90 {np.percentile(first - start, 90):.0f} max {(first - start).max():.0f}")
print(f"wave life: median {np.median(life):.0f}; spin share of life: median {np.median(spin / life):.3f} mean {np.mean(spin / life):.3f}")
base = r0.min()
print(f"realtime (us): starts {0:.2f}..{(r0.max() - base) / 100:.2f}; ends {(r1.min() - base) / 100:.2f}..{(r1.max() - base) / 100:.2f} median {(np.median(r1) - base) / 100:.2f}")
wg = np.arange(len(st)) // 16
cu_end = np.array([r1[wg == g].max() for g in np.unique(wg)]) - base
cu_first_end = np.array([r1[wg == g].min() for g in np.unique(wg)]) - base
print(f"per-CU (workgroup) end (us): min {cu_end.min()/100:.2f} median {np.median(cu_end)/100:.2f} max {cu_end.max()/100:.2f}; "
      f"spread inside a CU (last - first wave end): median {np.median(cu_end - cu_first_end)/100:.2f}")
clk = life / ((r1 - r0) / 100e6) / 1e9
print(f"clock (GHz): median {np.median(clk):.3f}")

# Where the SIMD-cycles go: hw_id (gfx9 HW_REG_HW_ID) bits 5:4 = SIMD; workgroup
# b runs on XCD b % 8 (round-robin dispatch).  Per SIMD: idle before its first
# task (from the kernel's first wave start) and after its last wave ends (to
# the kernel's last wave end), in us of realtime.
hw = st[:, 7]
simd = (hw >> 4) & 3
kend = r1.max()
first_rt = r0 + (first - start) / np.maximum(clk, 1e-3) / 10.0  # cycles -> 10 ns ticks
lead, tail, cu_tail, simd_spread = [], [], [], []
for g in np.unique(wg):
    sel = wg == g
    cu_e = r1[sel].max()
    cu_tail.append((kend - cu_e) / 100)
    ends = []
    for s in range(4):
        ss = sel & (simd == s)
        if not ss.any():
            continue
        lead.append((first_rt[ss].min() - base) / 100)
        e = r1[ss].max()
        ends.append(e)
        tail.append((kend - e) / 100)
    simd_spread.append((max(ends) - min(ends)) / 100)
lead, tail = np.array(lead), np.array(tail)
span = (kend - base) / 100
print(f"span {span:.2f} us; per SIMD: lead-in (first task) mean {lead.mean():.2f} us, "
      f"tail (idle after its last wave) mean {tail.mean():.2f} us "
      f"= {100 * (lead.mean() + tail.mean()) / span:.1f} % of the span")
print(f"  CU tail (kernel end - CU end) mean {np.mean(cu_tail):.2f} us; SIMD end spread inside a CU "
      f"median {np.median(simd_spread):.2f} p90 {np.percentile(simd_spread, 90):.2f} us")
xcd = np.unique(wg) % 8
cu_e = np.array([r1[wg == g].max() for g in np.unique(wg)]) - base
for x in range(8):
    sx = np.isin(wg, np.unique(wg)[xcd == x])
    print(f"  XCD {x}: clock {np.median(clk[sx]):.3f} GHz, CU end median {np.median(cu_e[xcd == x]) / 100:.2f} "
          f"max {cu_e[xcd == x].max() / 100:.2f} us, tasks {ntask[sx].sum()}")
