#!/usr/bin/env python3
"""SSD search timing on resident frames, for A/B runs of the matrix-core paths.

Times me_full_search_batch_device (SSD) on bench.py's 16-frame batches of the
1080p +-32 and 4K +-64 configs, F frames per call (one launch, or a prepass +
main launch pair), after a clock ramp, with HIP events on the launch stream;
checks the last call's fields against the committed per-frame pins (the
unmodified reference's ref_dump).  Prints one JSON line per (config, F).
The kernel path is whatever the loaded library plans (tuning build:
ME_HIP_LIB=libme_hip_tune.so ME_MFMA_S2K=0|1).
usage: python3 tools/ssd_ab.py [--frames 1,16] [--configs 1080p,4k] [--tag A]"""
import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import motionestimation_amd as me  # noqa: E402
from motionestimation_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", default="1,16")
    ap.add_argument("--configs", default="1080p,4k")
    ap.add_argument("--tag", default="")
    ap.add_argument("--ms", type=float, default=300.0, help="timed wall per (config, F)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    eng = me.Engine(devices=[0])
    for cfg_name in a.configs.split(","):
        cfg, blk, span = bench.CONFIGS[cfg_name]
        frames = bench.batch_frames(*synth.named_pair(cfg), 16)
        h, w = frames[0][0].shape
        nb = me.num_blocks(w, h, blk)
        pins = bench.load_pins(cfg_name, blk, span, "ssd")
        for F in (int(x) for x in a.frames.split(",")):
            ref_t = torch.from_numpy(np.stack([r for r, _ in frames[:F]])).to(dev)
            cur_t = torch.from_numpy(np.stack([c for _, c in frames[:F]])).to(dev)
            mv = torch.empty((F * nb, 2), dtype=torch.int16, device=dev)
            co = torch.empty(F * nb, dtype=torch.int32, device=dev)
            run = eng.prepared_batch_search(ref_t, 0, cur_t, 0, w, h, blk, span, "ssd", 0,
                                            (h + blk - 1) // blk, mv, co)
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.15:  # clock ramp
                for _ in range(4):
                    run()
                torch.cuda.synchronize()
            reps = 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < a.ms / 1e3:
                for _ in range(4):
                    run()
                reps += 4
                torch.cuda.synchronize()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            eng.device_check()
            fields = bench.batch_fields(mv, co, F)
            eq = sum(hashlib.sha256(bench.record_stream(m, c, w, h, blk, "ssd")).hexdigest() == pins[f]
                     for f, (m, c) in enumerate(fields))
            print(json.dumps({"tag": a.tag, "config": cfg_name, "frames": F, "ms_per_call": ms,
                              "us_per_frame": ms * 1e3 / F, "calls": reps,
                              "pinned_equal": eq, "pinned": F}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
