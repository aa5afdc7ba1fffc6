#!/usr/bin/env python3
"""Per-phase cycles of the band-walk SSD kernel (me_band.hip) from the
ME_STAMPS build (libme_hip_stamps.so): for every workgroup and wave, s_memtime
cycles summed over its iterations per phase [prologue, entries, fetch, tiles,
band end, producer, barrier wait].  Diagnostic only: the stamps cost time, so
absolute numbers are never quoted, only shares.
usage: python3 tools/bw_stamps.py [1080p|4k] [frames]"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from motionestimation_amd import _lib, synth  # noqa: E402
_lib.LIB_PATH = os.path.join(REPO, "motionestimation_amd", "lib", "libme_hip_stamps.so")
import bench  # noqa: E402
import motionestimation_amd as me  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "1080p"
F = int(sys.argv[2]) if len(sys.argv) > 2 else 16
_, blk, span = bench.CONFIGS[cfg]
frames = bench.batch_frames(*synth.named_pair(cfg), F)
h, w = frames[0][0].shape
nb = me.num_blocks(w, h, blk)
dev = torch.device("cuda", 0)
eng = me.Engine(devices=[0])
rt = torch.from_numpy(np.stack([r for r, _ in frames])).to(dev)
ct = torch.from_numpy(np.stack([c for _, c in frames])).to(dev)
mv = torch.empty((F * nb, 2), dtype=torch.int16, device=dev)
co = torch.empty(F * nb, dtype=torch.int32, device=dev)
for _ in range(20):
    eng.search_batch_device(rt, 0, ct, 0, w, h, blk, span, "ssd", 0, (h + blk - 1) // blk, mv, co)
torch.cuda.synchronize()
L = _lib.lib()
L.me_debug_bw_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
NW = 16  # stamp slots per workgroup (me_band.hip BW_STW)
buf = np.zeros(NW * 8 * 4096, np.uint64)
L.me_debug_bw_stamps(buf.ctypes.data, buf.size)
st = buf.reshape(4096, NW, 8).astype(np.float64)
used = st[:, 0, 7] > 0
st = st[used]
names = ["prologue", "entries", "fetch", "tiles", "band end", "producer", "barrier"]
nw = int((st[:, :, 7] > 0).any(axis=0).sum())  # waves of the kernel
st = st[:, :nw]
tot = st[:, :, :7].sum(axis=2)
print(f"{cfg} F={F}: {used.sum()} workgroups, iterations median {np.median(st[:, 0, 7]):.0f}")
print(f"  wave-lifetime cycles (stamped): median {np.median(tot):.0f}")
for k, nm in enumerate(names):
    share = st[:, :, k].sum() / tot.sum()
    per_it = np.median(st[:, :, k] / np.maximum(st[:, :, 7], 1))
    print(f"  {nm:9s} {100 * share:5.1f} %  median per iteration {per_it:8.1f} cycles")
for wv in range(nw):
    row = " ".join(f"{np.median(st[:, wv, k] / np.maximum(st[:, wv, 7], 1)):7.0f}" for k in range(1, 7))
    print(f"  wave {wv}: per iteration [entries fetch tiles end producer barrier] {row}")
# producers (the last 4 waves): per-WG totals [slot wait, DMA wait, hb S2,
# publish, production, hb search]
print("  producer totals per workgroup (median cycles): slot-wait, DMA-wait, hb-S2, publish, production, hb-search")
for wv in range(max(0, nw - 4), nw):
    row = " ".join(f"{np.median(st[:, wv, k]):8.0f}" for k in (1, 2, 3, 4, 5, 6))
    print(f"    wave {wv}: {row}")
# per-workgroup lifetime (the longest wave) by bands walked: which segments
# (top: fewer bands; bottom: + the partial row) end last
life = tot.max(axis=1)
print(f"  workgroup lifetime: median {np.median(life):.0f}  p90 {np.percentile(life, 90):.0f}  max {life.max():.0f}")
for it in sorted(set(st[:, 0, 7].astype(int))):
    sel = st[:, 0, 7].astype(int) == it
    print(f"    {it:3d} bands: {sel.sum():4d} workgroups, lifetime median {np.median(life[sel]):.0f} max {life[sel].max():.0f}")
    prod = " ".join(f"{np.median(st[sel][:, max(0, nw - 4):nw, k]):8.0f}" for k in (1, 2, 3, 4, 5, 6))
    print(f"        producers (slot-wait, DMA-wait, hb-S2, publish, production, hb-search): {prod}")

# absolute times (s_memrealtime, 100 MHz) of the last launch: workgroup start
# stagger and end spread, relative to the first workgroup's start
L.me_debug_bw_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
tb = np.zeros(NW * 2 * 4096, np.uint64)
L.me_debug_bw_times(tb.ctypes.data, tb.size)
tt = tb.reshape(4096, NW, 2)[used][:, :nw].astype(np.float64)
t0 = tt[:, :, 0].min()
starts = (tt[:, :, 0].min(axis=1) - t0) / 100.0  # us
ends = (tt[:, :, 1].max(axis=1) - t0) / 100.0
print(f"  workgroup start (us after the first): median {np.median(starts):.2f} p90 {np.percentile(starts, 90):.2f} max {starts.max():.2f}")
print(f"  workgroup end   (us after the first start): min {ends.min():.2f} median {np.median(ends):.2f} p90 {np.percentile(ends, 90):.2f} max {ends.max():.2f}")
