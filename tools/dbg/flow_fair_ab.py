"""A/B of flow-kernel settings in the tuning build (diagnostic): per-frame time of
back-to-back single-frame 1080p +-32 SAD searches and of 8-frame batches, after a
clock ramp, plus batch == single parity.  Settings come from the environment
(ME_FAIR, ME_FLOW_ONE, ...; ME_HIP_LIB=libme_hip_tune.so)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import motionestimation_amd as me  # noqa: E402
from motionestimation_amd import synth  # noqa: E402

F = int(os.environ.get("AB_FRAMES", "8"))
ref, cur = synth.named_pair("1080p")
h, w = ref.shape
nb = me.num_blocks(w, h, 16)
eng = me.Engine(devices=[0])
rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
# frames differ: frame f is the pair shifted 37 f columns (as bench.py does)
rb = torch.from_numpy(np.stack([np.roll(ref, 37 * f, axis=1) for f in range(F)])).cuda()
cb = torch.from_numpy(np.stack([np.roll(cur, 37 * f, axis=1) for f in range(F)])).cuda()
mv1 = torch.empty((nb, 2), dtype=torch.int16, device="cuda")
co1 = torch.empty(nb, dtype=torch.int32, device="cuda")
mvb = torch.empty((F * nb, 2), dtype=torch.int16, device="cuda")
cob = torch.empty(F * nb, dtype=torch.int32, device="cuda")


def single_all():
    for f in range(F):
        eng.full_search_device(rb[f], cb[f], 16, 32, "sad", mvb[f * nb:(f + 1) * nb], cob[f * nb:(f + 1) * nb])


def batch():
    eng.search_batch_device(rb, 0, cb, 0, w, h, 16, 32, "sad", 0, 68, mvb, cob)


def window(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3 / F


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:  # clock ramp
    batch()
    torch.cuda.synchronize()
single_all()
torch.cuda.synchronize()
ref_mv, ref_co = mvb.clone(), cob.clone()
batch()
torch.cuda.synchronize()
parity = bool(torch.equal(ref_mv, mvb) and torch.equal(ref_co, cob))
out = {k: os.environ.get(k) for k in ("ME_FAIR", "ME_FAIR_T", "ME_FLOW_ONE", "ME_FLOW_SLOTS") if os.environ.get(k)}
out["frames"] = F
out["single_us"] = [round(window(single_all, 20), 2) for _ in range(3)]
out["batch_us"] = [round(window(batch, 20), 2) for _ in range(3)]
out["parity"] = parity
print(json.dumps(out), flush=True)
