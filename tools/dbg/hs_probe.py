"""bench.host_stream (pinned 1080p pan, 64 pairs) after different preludes, to
find what makes the leg slower inside bench.py than alone.
usage: python3 tools/dbg/hs_probe.py <prelude>   (none | batch | cpu | both, each
optionally + "_stream": torch's current stream a created one, as in bench.py)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

import bench
import motionestimation_amd as me
from motionestimation_amd import synth

mode = sys.argv[1] if len(sys.argv) > 1 else "none"
dev = torch.device("cuda", 0)
if mode.endswith("_stream"):
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    mode = mode[:-7]
eng = me.Engine(devices=[0])
ref, cur = synth.frame_pair(1920, 1080, 1, 3, -3)
if mode in ("batch", "both"):
    frames = bench.batch_frames(ref, cur, 16)
    rt = torch.from_numpy(np.stack([r for r, _ in frames])).to(dev)
    ct = torch.from_numpy(np.stack([c for _, c in frames])).to(dev)
    nb = me.num_blocks(1920, 1080, 16)
    mv = torch.empty((16 * nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(16 * nb, dtype=torch.int32, device=dev)
    run = eng.prepared_batch_search(rt, 0, ct, 0, 1920, 1080, 16, 32, "sad", 0, 68, mv, co)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        run()
    torch.cuda.synchronize()
if mode in ("cpu", "both"):
    bench.cpu_baselines(ref, cur, 16, 32, "sad", None, 33188832)
for i in range(3):
    out = bench.host_stream(eng, 1920, 1080, 16, 32, "sad", 1, 3, -3, 0.07, 0.062, 33188832, 100.0)
    print(mode, i, round(out["pinned"]["pairs_per_s"]), round(out["pageable"]["pairs_per_s"]), flush=True)
eng.close()
