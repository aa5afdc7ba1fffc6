"""Does the pair pipeline's H2D traffic slow the search kernel?  Times a
batched 1080p SAD search of F frames (one launch, HIP events on the search
stream) alone and while a second stream keeps copying pinned 2 MB frames to
the device, as me_search_pairs' copy stream does.
usage: python3 tools/dbg/copy_interference.py [F ...]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

import motionestimation_amd as me
from motionestimation_amd import synth

W, H, B, S = 1920, 1080, 16, 32
dev = torch.device("cuda", 0)
eng = me.Engine(devices=[0])
nb = me.num_blocks(W, H, B)
host = me.pinned_frames(8, H, W)
synth.sequence(W, H, 8, 1, 3, -3, out=host)
host_t = [torch.from_numpy(host[i]) for i in range(8)]
dst = [torch.empty((H, W), dtype=torch.uint8, device=dev) for _ in range(8)]
cs = torch.cuda.Stream()
ss = torch.cuda.Stream()

for F in [int(a) for a in sys.argv[1:]] or [1, 4, 8, 16]:
    frames = [synth.frame_pair(W, H, 5 + f, 3, -3) for f in range(F)]
    rt = torch.from_numpy(np.stack([r for r, _ in frames])).to(dev)
    ct = torch.from_numpy(np.stack([c for _, c in frames])).to(dev)
    mv = torch.empty((F * nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(F * nb, dtype=torch.int32, device=dev)
    nby = (H + B - 1) // B

    def run(with_copies, reps=20):
        # warm clock: ~100 ms of back-to-back searches first (bench.py's ramp),
        # then reps searches back to back, each timed by its own events
        import time
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.1:
            eng.search_batch_device(rt, 0, ct, 0, W, H, B, S, "sad", 0, nby, mv, co,
                                    stream=ctypes.c_void_p(ss.cuda_stream))
            torch.cuda.synchronize()
        if with_copies:  # back-to-back 2 MB uploads on their own stream, longer than the searches
            with torch.cuda.stream(cs):
                for k in range(int(reps * F * 75 / 42) + 8):
                    dst[k % 8].copy_(host_t[k % 8], non_blocking=True)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record(ss)
        for i in range(reps):
            eng.search_batch_device(rt, 0, ct, 0, W, H, B, S, "sad", 0, nby, mv, co,
                                    stream=ctypes.c_void_p(ss.cuda_stream))
            ev[i + 1].record(ss)
        torch.cuda.synchronize()
        ts = sorted(ev[i].elapsed_time(ev[i + 1]) * 1e3 / F for i in range(reps))
        return ts[len(ts) // 2]

    run(False, 5)
    a = run(False)
    b = run(True)
    c = run(False)
    print(f"F={F}: us per frame alone {a:.1f} / {c:.1f}, with concurrent H2D {b:.1f}", flush=True)
