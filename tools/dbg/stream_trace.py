"""Streaming leg alone (bench.host_stream's pinned case) for a rocprofv3 timeline."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import motionestimation_amd as me
from motionestimation_amd import synth

# args: [npairs [width height]]
npairs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
eng = me.Engine(devices=[0])
pinned = me.pinned_frames(npairs + 1, h, w)
synth.sequence(w, h, npairs + 1, 1, 3, -3, out=pinned)
pairs = [(k, k + 1) for k in range(npairs)]
frames = list(pinned)
eng.search_pairs(frames, pairs, 16, 32, "sad")
torch.cuda.synchronize()
t0 = time.perf_counter()  # clock ramp, as bench.host_stream does (--ramp-ms 100)
while time.perf_counter() - t0 < 0.1:
    eng.search_pairs(frames, pairs, 16, 32, "sad")
for rep in range(int(os.environ.get("REPS", "3"))):  # REPS: more timed calls (outlier hunts)
    t0 = time.perf_counter()
    eng.search_pairs(frames, pairs, 16, 32, "sad")
    dt = time.perf_counter() - t0
    print(f"{w}x{h} {npairs} pairs: {dt*1e3:.3f} ms, {npairs/dt:.0f} pairs/s", flush=True)
