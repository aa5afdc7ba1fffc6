"""A/B of the SSD batch path (diagnostic, tuning build): per-frame time of F
frames searched in one me_full_search_batch_device call against the same F
frames one me_full_search_device call each, after a clock ramp; batch ==
single parity.  ME_MFMA_BATCH=0 turns the shared launches off."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import motionestimation_amd as me  # noqa: E402
from motionestimation_amd import synth  # noqa: E402

F = int(os.environ.get("AB_FRAMES", "16"))
cfg = os.environ.get("AB_CONFIG", "1080p")
blk, span = {"1080p": (16, 32), "4k": (16, 64)}[cfg]
ref, cur = synth.named_pair(cfg)
h, w = ref.shape
nb = me.num_blocks(w, h, blk)
nby = (h + blk - 1) // blk
eng = me.Engine(devices=[0])
rb = torch.from_numpy(np.stack([np.roll(ref, 37 * f, axis=1) for f in range(F)])).cuda()
cb = torch.from_numpy(np.stack([np.roll(cur, 37 * f, axis=1) for f in range(F)])).cuda()
mvb = torch.empty((F * nb, 2), dtype=torch.int16, device="cuda")
cob = torch.empty(F * nb, dtype=torch.int32, device="cuda")
mvs = torch.empty_like(mvb)
cos = torch.empty_like(cob)


def single_all():
    for f in range(F):
        eng.full_search_device(rb[f], cb[f], blk, span, "ssd", mvs[f * nb:(f + 1) * nb], cos[f * nb:(f + 1) * nb])


def batch():
    eng.search_batch_device(rb, 0, cb, 0, w, h, blk, span, "ssd", 0, nby, mvb, cob)


def window(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3 / F


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    batch()
    torch.cuda.synchronize()
single_all()
batch()
torch.cuda.synchronize()
out = {k: os.environ.get(k) for k in ("ME_MFMA_BATCH",) if os.environ.get(k)}
out.update(config=cfg, frames=F, parity=bool(torch.equal(mvs, mvb) and torch.equal(cos, cob)))
out["single_us"] = [round(window(single_all, 10), 2) for _ in range(3)]
out["batch_us"] = [round(window(batch, 10), 2) for _ in range(3)]
print(json.dumps(out), flush=True)
