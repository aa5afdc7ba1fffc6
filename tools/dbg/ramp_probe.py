"""Kernel time against time since the process started loading the GPU
(diagnostic): windows of back-to-back single-frame 1080p +-32 SAD searches,
then windows of the batched 8-frame search, then single frames again."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import motionestimation_amd as me  # noqa: E402
from motionestimation_amd import synth  # noqa: E402

ref, cur = synth.named_pair("1080p")
h, w = ref.shape
nb = me.num_blocks(w, h, 16)
eng = me.Engine(devices=[0])
mv = torch.empty((8 * nb, 2), dtype=torch.int16, device="cuda")
co = torch.empty(8 * nb, dtype=torch.int32, device="cuda")
rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
rb = torch.from_numpy(np.stack([ref] * 8)).cuda()
cb = torch.from_numpy(np.stack([cur] * 8)).cuda()
t0 = time.perf_counter()


def window(fn, n, per):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3 / per, 2)


single = lambda: eng.full_search_device(rt, ct, 16, 32, "sad", mv[:nb], co[:nb])  # noqa: E731
batch = lambda: eng.search_batch_device(rb, 0, cb, 0, w, h, 16, 32, "sad", 0, 68, mv, co)  # noqa: E731
out = {"single_us": [], "batch8_us_per_frame": [], "single_after_us": []}
for _ in range(40):
    out["single_us"].append(window(single, 50, 1))
for _ in range(20):
    out["batch8_us_per_frame"].append(window(batch, 6, 8))
for _ in range(20):
    out["single_after_us"].append(window(single, 50, 1))
time.sleep(1.0)
out["single_after_1s_idle_us"] = [window(single, 50, 1) for _ in range(10)]
out["elapsed_s"] = round(time.perf_counter() - t0, 3)
print(json.dumps(out))
eng.close()
