"""Pinned and pageable streaming rates over 16 and 64 1080p pairs."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import motionestimation_amd as me
from motionestimation_amd import synth

w, h = 1920, 1080
eng = me.Engine(devices=[0])
for npairs in (16, 64):
    pinned = me.pinned_frames(npairs + 1, h, w)
    synth.sequence(w, h, npairs + 1, 1, 3, -3, out=pinned)
    pageable = np.array(pinned)
    pairs = [(k, k + 1) for k in range(npairs)]
    for name, fr in (("pinned", list(pinned)), ("pageable", list(pageable))):
        eng.search_pairs(fr, pairs, 16, 32, "sad")
        torch.cuda.synchronize()
        ts = []
        for rep in range(5):
            t0 = time.perf_counter()
            eng.search_pairs(fr, pairs, 16, 32, "sad")
            ts.append(time.perf_counter() - t0)
        ts.sort()
        print(f"{npairs} {name}: median {npairs/ts[2]:.0f} pairs/s, worst {npairs/ts[-1]:.0f}", flush=True)
