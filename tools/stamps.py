#!/usr/bin/env python3
"""Per-workgroup timeline of the qsad kernel from the ME_STAMPS diagnostic
build (libme_hip_stamps.so): staging / compute / epilogue shares, per-CU
concurrency and the tail.  Diagnostic only: its absolute time is not quoted.
usage: python3 tools/stamps.py [1080p|4k|8k] [r0:r1 (one stripe's block rows)]"""
import ctypes, os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from motionestimation_amd import _lib, synth
_lib.LIB_PATH = os.path.join(REPO, "motionestimation_amd", "lib", "libme_hip_stamps.so")
import motionestimation_amd as me

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
for _ in range(5):
    if rows:  # one stripe, planes resident whole (row offsets 0)
        r0_, r1_ = (int(x) for x in rows.split(":"))
        eng.search_stripe_device(rt, 0, ct, 0, w, h, blk, span, "sad", r0_, r1_, mv, co)
    else:
        eng.full_search_device(rt, ct, blk, span, "sad", mv, co)
torch.cuda.synchronize()
L = _lib.lib()
L.me_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(8 << 16, np.uint64)
L.me_debug_stamps(buf.ctypes.data, buf.size)
st = buf.reshape(-1, 8)
st = st[st[:, 0] > 0]
hw = st[:, 4].astype(np.int64)
xcc = st[:, 5].astype(np.int64) & 0xF
# each XCD has its own s_memtime base: normalise per XCD to its first start
t0 = np.array([st[xcc == x, 0].min() for x in xcc], dtype=np.uint64)
s0, s1, s2, s3 = [(st[:, i] - t0).astype(np.float64) for i in range(4)]
cu = (xcc << 12) | ((hw >> 8) & 0xF) << 4 | (hw >> 13) & 0x7  # (xcc, cu_id, se_id)
items = st[:, 1].astype(np.int64)
dur = (st[:, 3] - st[:, 0]).astype(np.float64)
print(f"{cfg}: {len(st)} persistent workgroups, items per WG min {items.min()} max {items.max()}")
print(f"  WG lifetime cycles: min {dur.min():.0f} median {np.median(dur):.0f} max {dur.max():.0f}")
print(f"  lifetime per item: median {np.median(dur / np.maximum(items, 1)):.0f}")
stg = (st[:, 2] - st[:, 0]).astype(np.float64)
print(f"  start -> first item staged (cycles): median {np.median(stg):.0f} p90 {np.percentile(stg, 90):.0f} max {stg.max():.0f}")
for n in sorted(set(items.tolist())):
    sel = items == n
    print(f"  {n} items: {sel.sum()} WGs, median lifetime {np.median(dur[sel]):.0f}")

# per-CU load: HW_ID = cu_id[11:8] sh_id[12] se_id[15:13]; XCC from HW_REG_XCC_ID
cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
ucu, inv = np.unique(cu, return_inverse=True)
tot = np.bincount(inv, weights=items)
nwg = np.bincount(inv)
endt = np.array([(st[inv == i, 3] - t0[inv == i]).max() for i in range(len(ucu))], dtype=np.float64)
print(f"  CUs {len(ucu)}: WGs per CU {np.bincount(nwg)[1:]} (index = count-1)")
print(f"  items per CU min {tot.min():.0f} max {tot.max():.0f} mean {tot.mean():.2f}")
for n in sorted(set(tot.tolist())):
    sel = tot == n
    print(f"    {n:.0f} items: {sel.sum()} CUs, finish median {np.median(endt[sel]):.0f} max {endt[sel].max():.0f}")

# global timeline from s_memrealtime (100 MHz, chip-wide)
r0, r1 = st[:, 6].astype(np.int64), st[:, 7].astype(np.int64)
base = r0.min()
print(f"  realtime: starts {0:.0f}..{(r0.max()-base)*10:.0f} ns, ends {(r1.min()-base)*10:.0f}..{(r1.max()-base)*10:.0f} ns")
print("  start-time histogram (us):", np.histogram((r0 - base) / 100.0, bins=10)[0].tolist())
print("  end-time histogram (us):  ", np.histogram((r1 - base) / 100.0, bins=10)[0].tolist(),
      "edges", np.round(np.histogram((r1 - base) / 100.0, bins=10)[1], 1).tolist())
cu_end = np.array([r1[inv == i].max() for i in range(len(ucu))]) - base
cu_start = np.array([r0[inv == i].min() for i in range(len(ucu))]) - base
print(f"  per-CU busy span (us): start max {cu_start.max()/100:.1f}, end min {cu_end.min()/100:.1f} median {np.median(cu_end)/100:.1f} max {cu_end.max()/100:.1f}")
clk = (st[:, 3] - st[:, 0]).astype(np.float64) / ((r1 - r0).astype(np.float64) / 100e6) / 1e9
print(f"  shader clock during WG lifetime (GHz): median {np.median(clk):.3f} min {clk.min():.3f} max {clk.max():.3f}")
