#!/usr/bin/env python3
"""Host cost of one stripe-mode step on one GPU (diagnostic).

At N = 8 a 1080p stripe searches in ~16-19 us of GPU time, so the step can be
bound by the host: the ctypes search launch plus the RCCL gather call.  This
times, for one rank's stripe of an N-way split on ONE GPU, K back-to-back steps
of (a) the search alone, (b) search + async RCCL gather (double-buffered
records, as bench.py's StripeRun) in a world-size-1 RCCL group, and (c) the
gather alone, (d) search + the library's gather (me_gather_device, as
bench.py's RCCL ranks), and prints one JSON line per case: wall us per step against HIP-event us per step.

  python tools/step_overhead.py [--config 1080p] [--ways 8] [--rank 1] [--steps 2000]
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
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import bench
    import motionestimation_amd as me
    from motionestimation_amd import shard, synth

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    cfg, blk, span = bench.CONFIGS[a.config]
    w, h, seed, sx, sy = synth.CONFIGS[cfg]
    ref, cur = synth.frame_pair(w, h, seed, sx, sy)
    st = shard.plan(w, h, blk, span, a.ways)[a.rank]
    eng = me.Engine(devices=[0])
    ref_t = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).to(dev)
    cur_t = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).to(dev)
    recs = [torch.zeros((2, st.max_blocks), dtype=torch.int32, device=dev) for _ in range(2)]
    bufs = [[torch.empty_like(r)] for r in recs]
    works = [None, None]
    state = {"i": 0}

    def search(rec):
        mv = rec[0].view(torch.int16).view(st.max_blocks, 2)
        eng.search_stripe_device(ref_t, st.ref_y0, cur_t, st.cur_y0, w, h, blk, span, "sad",
                                 st.row_begin, st.row_end, mv, rec[1])

    def step_search():
        search(recs[0])

    def step_gather():
        k = state["i"] & 1
        state["i"] += 1
        if works[k] is not None:
            works[k].wait()
            works[k] = None
        search(recs[k])
        works[k] = dist.gather(recs[k], bufs[k], dst=0, async_op=True)

    def drain():
        for k in range(2):
            if works[k] is not None:
                works[k].wait()
                works[k] = None

    def run(name, fn, steps, finish=None):
        for _ in range(50):
            fn()
        if finish:
            finish()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(steps):
            fn()
        t_host = time.perf_counter() - t0
        if finish:
            finish()
        e1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(json.dumps({"case": name, "config": a.config, "ways": a.ways, "rank": a.rank,
                          "block_rows": st.row_end - st.row_begin, "steps": steps,
                          "wall_us_per_step": wall / steps * 1e6,
                          "host_enqueue_us_per_step": t_host / steps * 1e6,
                          "gpu_event_us_per_step": e0.elapsed_time(e1) / steps * 1e3}),
              flush=True)

    run("search", step_search, a.steps)
    run("search+gather", step_gather, a.steps, drain)

    def step_gather_only():
        k = state["i"] & 1
        state["i"] += 1
        if works[k] is not None:
            works[k].wait()
        works[k] = dist.gather(recs[k], bufs[k], dst=0, async_op=True)

    run("gather", step_gather_only, a.steps, drain)

    # (d) bench.py's RCCL path: the gather in libme_hip (me_gather_device) on a
    # side stream, ordered by events (a world-size-1 library communicator)
    eng.comm_init(eng.comm_unique_id(), 1, 0)
    gs = torch.cuda.Stream(dev)
    gs_h = ctypes.c_void_p(gs.cuda_stream)
    sev = [torch.cuda.Event() for _ in range(2)]
    gev = [torch.cuda.Event() for _ in range(2)]
    flat = [torch.empty((1,) + tuple(r.shape), dtype=r.dtype, device=dev) for r in recs]
    pend = [False, False]

    def step_libgather():
        k = state["i"] & 1
        state["i"] += 1
        cur_s = torch.cuda.current_stream()
        if pend[k]:
            cur_s.wait_event(gev[k])
        search(recs[k])
        sev[k].record(cur_s)
        gs.wait_event(sev[k])
        eng.gather_device(recs[k], flat[k], stream=gs_h)
        gev[k].record(gs)
        pend[k] = True

    def libdrain():
        for k in range(2):
            if pend[k]:
                torch.cuda.current_stream().wait_event(gev[k])
                pend[k] = False

    run("search+libgather", step_libgather, a.steps, libdrain)

    def step_libgather_same():  # the gather on the search's own stream, no events
        k = state["i"] & 1
        state["i"] += 1
        search(recs[k])
        eng.gather_device(recs[k], flat[k])

    run("search+libgather_same_stream", step_libgather_same, a.steps)

    # (e) bench.py's StripeRun: the same two calls, marshalled once
    mvs = [r[0].view(torch.int16).view(st.max_blocks, 2) for r in recs]
    ps = [eng.prepared_stripe_search(ref_t, st.ref_y0, cur_t, st.cur_y0, w, h, blk, span, "sad",
                                     st.row_begin, st.row_end, mvs[k], recs[k][1])
          for k in range(2)]
    pg = [eng.prepared_gather(recs[k], flat[k]) for k in range(2)]

    def step_prepared():
        k = state["i"] & 1
        state["i"] += 1
        ps[k]()
        pg[k]()

    run("prepared_search+libgather", step_prepared, a.steps)
    run("prepared_search", lambda: ps[0](), a.steps)
    torch.cuda.synchronize()
    ok = all(torch.equal(flat[k][0], recs[k]) for k in range(2))
    print(json.dumps({"case": "libgather_parity", "equal": ok}), flush=True)
    dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
