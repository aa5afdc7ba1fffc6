"""Per-launch fixed cost of the search kernel: time one launch on frames of
1x, 2x, 4x the 1080p height (same width, block, range) -- if the time per
candidate falls with size, launch ramp / drain / imbalance dominate."""
import argparse
import os
import sys
import json

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import motionestimation_amd as me
from motionestimation_amd import synth


def _stripe_candidates(me, w, h, blk, span, r0, r1):
    """Exact candidates of block rows [r0, r1) (main.c:73-76 clamping)."""
    nbx = (w + blk - 1) // blk
    tot = 0
    for by in range(r0, r1):
        tly = by * blk
        bh = min(blk, h - tly)
        ny = min(span, h - bh - tly) - max(-span, -tly) + 1
        for bx in range(nbx):
            tlx = bx * blk
            bw = min(blk, w - tlx)
            tot += (min(span, w - bw - tlx) - max(-span, -tlx) + 1) * ny
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cost", default="sad")
    ap.add_argument("--blk", type=int, default=16)
    ap.add_argument("--span", type=int, default=32)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--heights", default="1080,2160,4320")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rows", default="",
                    help="block rows r0:r1 -- time one row stripe (me_full_search_stripe_device)")
    a = ap.parse_args()
    eng = me.Engine()
    dev = torch.device("cuda", 0)
    for h in [int(x) for x in a.heights.split(",")]:
        ref, cur = synth.frame_pair(a.width, h, 1, 3, -3)
        r, c = torch.from_numpy(ref).to(dev), torch.from_numpy(cur).to(dev)
        nb = me.num_blocks(a.width, h, a.blk)
        mv = torch.empty((nb, 2), dtype=torch.int16, device=dev)
        co = torch.empty(nb, dtype=torch.int32, device=dev)
        nby = (h + a.blk - 1) // a.blk
        r0, r1 = (int(v) for v in a.rows.split(":")) if a.rows else (0, nby)

        def run():
            if a.rows:
                eng.search_stripe_device(r, 0, c, 0, a.width, h, a.blk, a.span, a.cost, r0, r1, mv, co)
            else:
                eng.full_search_device(r, c, a.blk, a.span, a.cost, mv, co)
        for _ in range(5):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        nbx = (a.width + a.blk - 1) // a.blk
        cand = me.candidate_count(a.width, h, a.blk, a.span) if not a.rows else \
            _stripe_candidates(me, a.width, h, a.blk, a.span, r0, r1)
        print(json.dumps({"width": a.width, "height": h, "cost": a.cost, "rows": [r0, r1], "ms": ms,
                          "cand_per_s": cand / ms * 1e3,
                          "ns_per_mcand": ms * 1e6 / (cand / 1e6)}), flush=True)


if __name__ == "__main__":
    main()
