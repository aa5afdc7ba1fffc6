"""Per-rank stripe search time on ONE GPU, for the N-GPU row-stripe split.

For N in --ranks, plan the N candidate-balanced stripes (me_plan_stripes) of a
BASELINE config and time every rank's stripe search (its halo-only planes,
me_full_search_stripe_device) back to back on this GPU.  The slowest stripe is
the compute-bound step time of the N-GPU strong-scaling run (before the
RCCL gather), so t(N=1) / max_r t_r(N) is the compute-side speed-up ceiling.
--frames F times a rank's F-frame step as bench.py runs it: stripe (r + f) % N
of frame f for rank r, all in one me_search_stripes_device call.
One JSON line per N (times per launch, i.e. per F frames).

  python tools/stripe_sweep.py [--config 1080p|4k|8k] [--cost sad] [--ranks 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import motionestimation_amd as me  # noqa: E402
from motionestimation_amd import shard, synth  # noqa: E402

CONFIGS = {"1080p": ("1080p", 16, 32), "4k": ("4k", 16, 64), "8k": ("8k", 8, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1080p", choices=list(CONFIGS))
    ap.add_argument("--cost", default="sad")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--frames", type=int, default=1,
                    help="frames per launch (me_full_search_batch_device): the batched step")
    a = ap.parse_args()
    cfg, blk, span = CONFIGS[a.config]
    w, h, seed, sx, sy = synth.CONFIGS[cfg]
    ref, cur = synth.frame_pair(w, h, seed, sx, sy)
    eng = me.Engine()
    # GPU clock ramp (bench.clock_ramp): ~100 ms of whole-frame searches first,
    # or the first (N = 1) line is timed on a rising clock
    rt0, ct0 = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
    nb0 = me.num_blocks(w, h, blk)
    mv0 = torch.empty((nb0, 2), dtype=torch.int16, device="cuda")
    co0 = torch.empty(nb0, dtype=torch.int32, device="cuda")
    t_end = time.perf_counter() + 0.1
    while time.perf_counter() < t_end:
        for _ in range(4):
            eng.full_search_device(rt0, ct0, blk, span, a.cost, mv0, co0)
        torch.cuda.synchronize()
    base = None
    F = a.frames
    frames = [(np.roll(ref, 37 * f, axis=1), np.roll(cur, 37 * f, axis=1)) for f in range(F)]
    for n in [int(x) for x in a.ranks.split(",")]:
        times = []
        plan = shard.plan(w, h, blk, span, n)
        for r in range(n):
            # rank r's step: stripe (r + f) % n of frame f (bench.py StripeRun)
            own = [plan[(r + f) % n] for f in range(F)]
            jobs, keep = [], []
            for f, st in enumerate(own):
                if not st.nblocks:
                    continue
                rt = torch.from_numpy(frames[f][0][st.ref_y0:st.ref_y1].copy()).cuda()
                ct = torch.from_numpy(frames[f][1][st.cur_y0:st.cur_y1].copy()).cuda()
                mv = torch.empty((st.nblocks, 2), dtype=torch.int16, device="cuda")
                co = torch.empty(st.nblocks, dtype=torch.int32, device="cuda")
                keep += [rt, ct, mv, co]
                jobs.append((rt, st.ref_y0, ct, st.cur_y0, st.row_begin, st.row_end, mv, co))
            if not jobs:
                times.append(0.0)
                continue
            run = eng.prepared_stripes_search(w, h, blk, span, a.cost, jobs, stride=w)
            # clock ramp before every timed window: allocating a rank's planes
            # leaves the GPU idle long enough for the clock to drop
            t_end = time.perf_counter() + 0.15
            while time.perf_counter() < t_end:
                for _ in range(4):
                    run()
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / a.iters)
        t = max(times)
        base = base or t
        print(json.dumps({"config": a.config, "cost": a.cost, "ranks": n, "frames": a.frames,
                          "stripe_ms": [round(x, 4) for x in times], "max_ms": t,
                          "compute_speedup_vs_1": base / t}), flush=True)


if __name__ == "__main__":
    main()
