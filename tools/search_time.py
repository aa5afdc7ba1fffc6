#!/usr/bin/env python3
"""Time one search per call on a resident synthetic pair (HIP events over
back-to-back calls, after a clock ramp) for A/B runs of library builds
(ME_HIP_LIB=...): prints one JSON line per (config, cost).
usage: python3 tools/search_time.py [--configs 8k] [--costs ssd] [--ms 400] [--tag A]
The fields are checked elsewhere (tests/test_gpu_fullframe.py pins the 8K
searches against the unmodified reference over every block); this line
carries a SHA-256 of the last call's records for cross-build comparison."""
import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
import motionestimation_amd as me  # noqa: E402
from motionestimation_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="8k")
    ap.add_argument("--costs", default="ssd")
    ap.add_argument("--ms", type=float, default=400.0)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    eng = me.Engine(devices=[0])
    for cfg_name in a.configs.split(","):
        cfg, blk, span = bench.CONFIGS[cfg_name]
        ref, cur = synth.named_pair(cfg)
        h, w = ref.shape
        nb = me.num_blocks(w, h, blk)
        rt, ct = torch.from_numpy(ref).to(dev), torch.from_numpy(cur).to(dev)
        mv = torch.empty((nb, 2), dtype=torch.int16, device=dev)
        co = torch.empty(nb, dtype=torch.int32, device=dev)
        for cost in a.costs.split(","):
            run = lambda: eng.full_search_device(rt, ct, blk, span, cost, mv, co)  # noqa: E731
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.15:
                run()
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 0
            e0.record()
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < a.ms / 1e3:
                run()
                reps += 1
                torch.cuda.synchronize()
            e1.record()
            torch.cuda.synchronize()
            eng.device_check()
            digest = hashlib.sha256(mv.cpu().numpy().tobytes() + co.cpu().numpy().tobytes()).hexdigest()[:16]
            print(json.dumps({"tag": a.tag, "config": cfg_name, "cost": cost,
                              "ms_per_call": e0.elapsed_time(e1) / reps, "calls": reps,
                              "path": me.last_search_path(), "records_sha": digest}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
