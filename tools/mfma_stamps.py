#!/usr/bin/env python3
"""Per-workgroup timeline of the MFMA SSD kernel from the ME_STAMPS build
(libme_hip_stamps.so): setup / chunk / tail shares, workgroups per CU at once.
Diagnostic only: its absolute time is never quoted.
usage: python3 tools/mfma_stamps.py [1080p|4k]"""
import ctypes, os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from motionestimation_amd import _lib, synth
_lib.LIB_PATH = os.path.join(REPO, "motionestimation_amd", "lib", "libme_hip_stamps.so")
import motionestimation_amd as me

cfg = sys.argv[1] if len(sys.argv) > 1 else "1080p"
blk, span = {"1080p": (16, 32), "4k": (16, 64)}[cfg]
ref, cur = synth.named_pair(cfg)
h, w = ref.shape
eng = me.Engine(devices=[0])
rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
n = me.num_blocks(w, h, blk)
mv = torch.empty((n, 2), dtype=torch.int16, device="cuda")
co = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(5):
    eng.full_search_device(rt, ct, blk, span, "ssd", mv, co)
torch.cuda.synchronize()
L = _lib.lib()
L.me_debug_mfma_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(8 << 14, np.uint64)
L.me_debug_mfma_stamps(buf.ctypes.data, buf.size)
st = buf.reshape(-1, 8)
st = st[st[:, 3] > 0]
hw = st[:, 4].astype(np.int64)
xcc = st[:, 5].astype(np.int64) & 0xF
rt0 = st[:, 6].astype(np.float64)
rt1 = st[:, 7].astype(np.float64)
base = rt0.min()
a, b = (rt0 - base) / 100.0, (rt1 - base) / 100.0  # s_memrealtime: 100 MHz -> us
print(f"{cfg}: {len(st)} workgroups; kernel span {b.max():.1f} us (realtime)")
print(f"  WG lifetime us: min {np.min(b - a):.2f} median {np.median(b - a):.2f} max {np.max(b - a):.2f}")
print(f"  start us: min {a.min():.2f} median {np.median(a):.2f} max {a.max():.2f}")
cyc = st[:, 3].astype(np.float64) - st[:, 0]
setup = st[:, 1].astype(np.float64) - st[:, 0]
ch0 = np.where(st[:, 2] > 0, st[:, 2].astype(np.float64) - st[:, 1], np.nan)
print(f"  cycles: lifetime median {np.median(cyc):.0f}, setup+stage0 median {np.median(setup):.0f}, "
      f"chunk0 compute median {np.nanmedian(ch0):.0f}")
print(f"  clock estimate (lifetime cycles / us): {np.median(cyc / np.maximum(b - a, 1e-3)):.0f} MHz")
cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
ucu, inv = np.unique(cu, return_inverse=True)
print(f"  CUs used {len(ucu)}; WGs per CU histogram {np.bincount(np.bincount(inv))[1:]}")
# max concurrent WGs on one CU
conc = []
for i in range(len(ucu)):
    sel = inv == i
    ev = sorted([(t, 1) for t in a[sel]] + [(t, -1) for t in b[sel]], key=lambda e: (e[0], e[1]))
    c = m = 0
    for _, d in ev:
        c += d
        m = max(m, c)
    conc.append(m)
print(f"  max concurrent WGs per CU: histogram {np.bincount(conc)[1:]}")

# prepass lifetimes (s_memtime per workgroup: start, end)
L.me_debug_prep_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
pb = np.zeros(6 << 14, np.uint64)
L.me_debug_prep_stamps(pb.ctypes.data, pb.size)
ps = pb.reshape(-1, 6)
full = ps[(ps[:, 3] > 0)].astype(np.float64)
print(f"prepass: {len(full)} main workgroups; lifetime cycles median {np.median(full[:, 3] - full[:, 0]):.0f}, "
      f"max {np.max(full[:, 3] - full[:, 0]):.0f}")
for nm, a0, a1 in (("loads + vertical sums (thread 0)", 0, 1), ("to the barrier", 1, 2), ("stores", 2, 3)):
    d = full[:, a1] - full[:, a0]
    print(f"  prepass {nm}: median {np.median(d):.0f} p90 {np.percentile(d, 90):.0f} cycles")
ra, rb = full[:, 4] - full[:, 4].min(), full[:, 5] - full[:, 4].min()
print(f"prepass realtime us: starts min {ra.min()/100:.2f} median {np.median(ra)/100:.2f} max {ra.max()/100:.2f}; "
      f"ends max {rb.max()/100:.2f}")
# slowest workgroups (tile index = blockIdx.x for the MFMA kernel)
ids = np.nonzero(buf.reshape(-1, 8)[:, 3] > 0)[0]
life = b - a
order = np.argsort(-life)[:12]
print("  slowest WGs (blockIdx, lifetime us):", [(int(ids[i]), round(float(life[i]), 1)) for i in order])

# block-major kernel: per band, wave 0's compute end and the barrier exit
try:
    L.me_debug_band_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    bs = np.zeros(32 << 12, np.uint64)
    L.me_debug_band_stamps(bs.ctypes.data, bs.size)
    bs = bs.reshape(-1, 32).astype(np.float64)
    mst = buf.reshape(-1, 8).astype(np.float64)
    rows = []
    for w in range(min(len(bs), len(mst))):
        if mst[w, 1] == 0 or bs[w, 0] == 0:
            continue
        t = [mst[w, 1]] + [v for v in bs[w] if v > 0]
        rows.append(np.diff(np.array(t)))
    if rows:
        n = max(len(r) for r in rows)
        full = [r for r in rows if len(r) == n]
        med = np.median(np.array(full), axis=0)
        print(f"bands: {len(full)} workgroups with {n // 2} bands; median cycles per band "
              f"[compute, barrier wait]: " + ", ".join(f"[{med[2*i]:.0f}, {med[2*i+1]:.0f}]" for i in range(n // 2)))
except AttributeError:
    pass
