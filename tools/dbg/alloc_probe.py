"""Does where the planes live change the 1080p search time?  (diagnostic)
Times the single-frame 1080p +-32 SAD search (HIP events, 100 back-to-back
launches) with ref / cur in: their own 2 MB torch tensors; slices of one large
tensor; slices of a batch tensor [8, H, W]; and the batched search of 8 frames."""
import json
import os
import sys

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


def timeit(fn, n=100):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def single(rt, ct):
    return timeit(lambda: eng.full_search_device(rt, ct, 16, 32, "sad", mv[:nb], co[:nb]))


out = {}
rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
out["own_2MB_tensors"] = single(rt, ct)
big = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
big[:h * w].copy_(torch.from_numpy(ref).view(-1))
big[128 << 20:(128 << 20) + h * w].copy_(torch.from_numpy(cur).view(-1))
out["slices_of_256MB"] = single(big[:h * w].view(h, w), big[128 << 20:(128 << 20) + h * w].view(h, w))
rb = torch.from_numpy(np.stack([ref] * 8)).cuda()
cb = torch.from_numpy(np.stack([cur] * 8)).cuda()
out["frame0_of_batch_tensor"] = single(rb[0], cb[0])
out["frame5_of_batch_tensor"] = single(rb[5], cb[5])
out["own_2MB_tensors_again"] = single(rt, ct)
out["batch8_per_frame"] = timeit(lambda: eng.search_batch_device(
    rb, 0, cb, 0, w, h, 16, 32, "sad", 0, (h + 15) // 16, mv, co), 20) / 8
print(json.dumps(out))
eng.close()
