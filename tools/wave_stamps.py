#!/usr/bin/env python3
"""Per-wave timeline of the persistent item kernel (me_fast_kernel) from the
ME_STAMPS diagnostic build: where each workgroup's waves sit (SIMD), when each
wave's first item is staged, when its task loop ends and when it exits.
Diagnostic only; absolute times are not quoted.

usage: python3 tools/wave_stamps.py [1080p|4k|8k] [r0:r1 (one stripe's block rows)]"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from motionestimation_amd import _lib, synth  # noqa: E402
_lib.LIB_PATH = os.path.join(REPO, "motionestimation_amd", "lib", "libme_hip_stamps.so")
import motionestimation_amd as me  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "1080p"
blk, span = {"1080p": (16, 32), "4k": (16, 64), "8k": (8, 128)}[cfg]
ref, cur = synth.named_pair(cfg)
h, w = ref.shape
eng = me.Engine(devices=[0])
rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
n = me.num_blocks(w, h, blk)
mv = torch.empty((n, 2), dtype=torch.int16, device="cuda")
co = torch.empty(n, dtype=torch.int32, device="cuda")
rows = sys.argv[2] if len(sys.argv) > 2 else ""
L = _lib.lib()
L.me_debug_wave_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(8 << 14, np.uint64)
for _ in range(5):
    L.me_debug_wave_stamps(buf.ctypes.data, 0)
    if rows:
        r0_, r1_ = (int(x) for x in rows.split(":"))
        eng.search_stripe_device(rt, 0, ct, 0, w, h, blk, span, "sad", r0_, r1_, mv, co)
    else:
        eng.full_search_device(rt, ct, blk, span, "sad", mv, co)
torch.cuda.synchronize()
L.me_debug_wave_stamps(buf.ctypes.data, buf.size)
st = buf.reshape(-1, 8)
valid = st[:, 0] > 0
idx = np.nonzero(valid)[0]
st = st[valid]
hw = st[:, 4].astype(np.int64)
xcc = st[:, 5].astype(np.int64) & 0xF
simd = (hw >> 4) & 3
cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
# workgroup -> XCD placement: the kernels assume blocks b and b + 8 share an
# XCD (bands of tiles per b % 8); print which XCCs each residue landed on
res = {}
for g_, x_ in zip(idx // 4, xcc):
    res.setdefault(int(g_) % 8, set()).add(int(x_))
print("  XCC ids per workgroup index % 8:", {r: sorted(v) for r, v in sorted(res.items())})
# per-XCD s_memtime base
base = {x: st[xcc == x, 0].min() for x in np.unique(xcc)}
b = np.array([base[x] for x in xcc], dtype=np.uint64)
t_start, t_staged, t_loop, t_end = [(st[:, i] - b).astype(np.float64) for i in range(4)]
wpg = 4  # waves per workgroup (256 threads)
wg = idx // wpg
print(f"{cfg} rows {rows or 'all'}: {len(st)} waves, {len(np.unique(wg))} workgroups, {len(np.unique(cu))} CUs")
print(f"  staged (cycles after wave start): median {np.median(t_staged - t_start):.0f} "
      f"p90 {np.percentile(t_staged - t_start, 90):.0f} max {(t_staged - t_start).max():.0f}")
print(f"  compute (staged -> loop end): median {np.median(t_loop - t_staged):.0f} "
      f"p10 {np.percentile(t_loop - t_staged, 10):.0f} p90 {np.percentile(t_loop - t_staged, 90):.0f}")
print(f"  loop end -> exit: median {np.median(t_end - t_loop):.0f} p90 {np.percentile(t_end - t_loop, 90):.0f}")
# SIMD placement of each workgroup's waves
spread = []
for g in np.unique(wg):
    spread.append(len(np.unique(simd[wg == g])))
print("  distinct SIMDs per workgroup:", np.bincount(spread).tolist(), "(index = count)")
# per CU: the workgroups ordered by staging time
ranks = {}
simd_busy = []
for c in np.unique(cu):
    sel = cu == c
    gs = np.unique(wg[sel])
    rows_ = sorted((t_staged[(wg == g)].max(), t_loop[(wg == g)].max(), t_end[(wg == g)].max(), g)
                   for g in gs)
    for r, (s_, l_, e_, g) in enumerate(rows_):
        ranks.setdefault(r, []).append((s_, l_, e_))
    # per SIMD: waves resident and busy span
    for s in range(4):
        ss = sel & (simd == s)
        if ss.any():
            simd_busy.append((ss.sum(), t_loop[ss].max() - t_staged[ss].min()))
print("  per-CU rank of workgroup (by staging): median [staged, loop end, exit] cycles")
for r in sorted(ranks):
    a = np.array(ranks[r])
    print(f"    rank {r}: n {len(a)}  staged {np.median(a[:, 0]):.0f}  loop end {np.median(a[:, 1]):.0f}  "
          f"exit {np.median(a[:, 2]):.0f}")
sb = np.array(simd_busy)
print("  waves per SIMD:", np.bincount(sb[:, 0].astype(int)).tolist())
print(f"  per-SIMD busy span (first staged -> last loop end): median {np.median(sb[:, 1]):.0f} "
      f"max {sb[:, 1].max():.0f}")
r0, r1 = st[:, 6].astype(np.int64), st[:, 7].astype(np.int64)
rb = r0.min()
print(f"  realtime: wave starts 0..{(r0.max() - rb) * 10} ns, exits {(r1.min() - rb) * 10}..{(r1.max() - rb) * 10} ns")
clk = (st[:, 3] - st[:, 0]).astype(np.float64) / ((r1 - r0).astype(np.float64) / 100e6) / 1e9
print(f"  clock (GHz): median {np.median(clk):.3f}")
eng.close()
