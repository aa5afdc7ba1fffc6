#!/usr/bin/env python3
"""Host cost of one stripe-mode step on one GPU (diagnostic).

At N = 8 a 1080p stripe searches in ~16-19 us of GPU time, so the step can be
bound by the host: the ctypes search launch plus the RCCL gather call.  This
times, for one rank's stripe of an N-way split on ONE GPU (a world-size-1
library communicator), K back-to-back steps of
  prepared_search            the search alone, arguments marshalled once
  prepared_search+libgather  search + me_gather_device on the same stream
                             (bench.py's direct path, --no-graph)
  graph_search               the search replayed from a captured hipGraph
  graph_search+libgather     search + gather in one graph (bench.py --graph)
  batchF_search              the rank's stripes of F frames (stripe (rank + f) % N
                             of frame f) in one me_search_stripes_device call
  batchF_search+libgather    ... and one gather of their records (bench.py's step)
and prints one JSON line per case: wall us per step, host enqueue us per step
and HIP-event us per step (batch cases: also per frame); then the gathered
records' parity.

  python tools/step_overhead.py [--config 1080p] [--ways 8] [--rank 1] [--steps 2000] [--frames 8]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1080p")
    ap.add_argument("--ways", type=int, default=8)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--cost", default="sad")
    ap.add_argument("--frames", type=int, default=8)
    a = ap.parse_args()
    import torch
    import bench
    import motionestimation_amd as me
    from motionestimation_amd import shard, synth

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))  # capturable
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cfg, blk, span = bench.CONFIGS[a.config]
    w, h, seed, sx, sy = synth.CONFIGS[cfg]
    ref, cur = synth.frame_pair(w, h, seed, sx, sy)
    st = shard.plan(w, h, blk, span, a.ways)[a.rank]
    eng = me.Engine(devices=[0])
    eng.comm_init(eng.comm_unique_id(), 1, 0)
    ref_t = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).to(dev)
    cur_t = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).to(dev)
    recs = [torch.zeros((2, st.max_blocks), dtype=torch.int32, device=dev) for _ in range(2)]
    flat = [torch.empty((1,) + tuple(r.shape), dtype=r.dtype, device=dev) for r in recs]
    mvs = [r[0].view(torch.int16).view(st.max_blocks, 2) for r in recs]
    ps = [eng.prepared_stripe_search(ref_t, st.ref_y0, cur_t, st.cur_y0, w, h, blk, span, a.cost,
                                     st.row_begin, st.row_end, mvs[k], recs[k][1])
          for k in range(2)]
    pg = [eng.prepared_gather(recs[k], flat[k]) for k in range(2)]
    state = {"i": 0}

    def run(name, fn, steps, frames=1):
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(steps):
            fn()
        t_host = time.perf_counter() - t0
        e1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        rec = {"case": name, "config": a.config, "cost": a.cost, "ways": a.ways,
               "rank": a.rank, "block_rows": st.row_end - st.row_begin, "frames": frames,
               "steps": steps, "wall_us_per_step": wall / steps * 1e6,
               "host_enqueue_us_per_step": t_host / steps * 1e6,
               "gpu_event_us_per_step": e0.elapsed_time(e1) / steps * 1e3}
        if frames > 1:
            rec["wall_us_per_frame"] = rec["wall_us_per_step"] / frames
        print(json.dumps(rec), flush=True)

    def alternate(calls):
        def step():
            k = state["i"] & 1
            state["i"] += 1
            for c in calls[k]:
                c()
        return step

    run("prepared_search", lambda: ps[0](), a.steps)
    run("prepared_search+libgather", alternate([(ps[0], pg[0]), (ps[1], pg[1])]), a.steps)
    gs = [eng.capture(stream, ps[k]) for k in range(2)]
    run("graph_search", gs[0].prepared(stream), a.steps)
    gg = [eng.capture(stream, lambda k=k: (ps[k](), pg[k]())) for k in range(2)]
    run("graph_search+libgather", alternate([(gg[0].prepared(stream),),
                                             (gg[1].prepared(stream),)]), a.steps)
    # bench.py's step: the rank's stripes of F frames in one call + one gather
    F = a.frames
    stripes = shard.plan(w, h, blk, span, a.ways)
    own = [stripes[(a.rank + f) % a.ways] for f in range(F)]
    mb = stripes[0].max_blocks
    ref_b = torch.zeros((F, max(o.ref_y1 - o.ref_y0 for o in own), w), dtype=torch.uint8, device=dev)
    cur_b = torch.zeros((F, max(o.cur_y1 - o.cur_y0 for o in own), w), dtype=torch.uint8, device=dev)
    for f, o in enumerate(own):
        ref_b[f, :o.ref_y1 - o.ref_y0] = torch.from_numpy(ref[o.ref_y0:o.ref_y1].copy())
        cur_b[f, :o.cur_y1 - o.cur_y0] = torch.from_numpy(cur[o.cur_y0:o.cur_y1].copy())
    brecs = [torch.zeros((2, F * mb), dtype=torch.int32, device=dev) for _ in range(2)]
    bflat = [torch.empty((1,) + tuple(r.shape), dtype=r.dtype, device=dev) for r in brecs]
    bmvs = [r[0].view(torch.int16).view(F * mb, 2) for r in brecs]
    bps = [eng.prepared_stripes_search(
        w, h, blk, span, a.cost,
        [(ref_b[f], o.ref_y0, cur_b[f], o.cur_y0, o.row_begin, o.row_end, bmvs[k][f * mb:],
          brecs[k][1][f * mb:]) for f, o in enumerate(own)], stride=w) for k in range(2)]
    bpg = [eng.prepared_gather(brecs[k], bflat[k]) for k in range(2)]
    run(f"batch{F}_search", lambda: bps[0](), max(a.steps // F, 50), F)
    run(f"batch{F}_search+libgather", alternate([(bps[0], bpg[0]), (bps[1], bpg[1])]),
        max(a.steps // F, 50), F)
    torch.cuda.synchronize()
    eng.device_check()
    ok = all(torch.equal(flat[k][0], recs[k]) for k in range(2))
    ok = ok and all(torch.equal(bflat[k][0], brecs[k]) for k in range(2))
    print(json.dumps({"case": "libgather_parity", "equal": ok}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
