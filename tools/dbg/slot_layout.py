"""Pair-pipeline kernel cost by frame layout: 8 consecutive pairs of a pan
(pair k = frames k, k + 1) searched in one job-table launch, frames in one
stacked tensor vs in separate allocations (the stream's slots), warm clock,
HIP events on one stream.  usage: python3 tools/dbg/slot_layout.py"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import motionestimation_amd as me
from motionestimation_amd import synth

W, H, B, S, F = 1920, 1080, 16, 32, 8
dev = torch.device("cuda", 0)
eng = me.Engine(devices=[0])
nb = me.num_blocks(W, H, B)
nby = (H + B - 1) // B
host = me.pinned_frames(F + 1, H, W)
synth.sequence(W, H, F + 1, 1, 3, -3, out=host)
stacked = torch.from_numpy(np.array(host)).to(dev)
separate = [torch.from_numpy(np.array(host[i])).to(dev) for i in range(F + 1)]
outs = [(torch.empty((nb, 2), dtype=torch.int16, device=dev), torch.empty(nb, dtype=torch.int32, device=dev))
        for _ in range(F)]
ss = torch.cuda.Stream()


def jobs_of(frames):
    return [(frames[k], 0, frames[k + 1], 0, 0, nby, outs[k][0], outs[k][1]) for k in range(F)]


def timed(jobs, reps=20):
    fn = eng.prepared_stripes_search(W, H, B, S, "sad", jobs, stream=ctypes.c_void_p(ss.cuda_stream))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        fn()
        torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    with torch.cuda.stream(ss):
        ev[0].record(ss)
        for i in range(reps):
            fn()
            ev[i + 1].record(ss)
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) * 1e3 / F for i in range(reps))
    return ts[len(ts) // 2]


for rep in range(2):
    a = timed(jobs_of([stacked[i] for i in range(F + 1)]))
    b = timed(jobs_of(separate))
    print(f"8 pan pairs per launch, us per pair: stacked frames {a:.1f}, separate allocations {b:.1f}", flush=True)
