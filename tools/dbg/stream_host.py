"""Per-pair host cost of me_search_pairs: tiny frames (kernel time negligible)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import motionestimation_amd as me
from motionestimation_amd import synth

for (w, h) in [(64, 64), (1920, 1080)]:
    for npairs in (16, 64):
        eng = me.Engine(devices=[0])
        pinned = me.pinned_frames(npairs + 1, h, w)
        synth.sequence(w, h, npairs + 1, 1, 3, -3, out=pinned)
        pairs = [(k, k + 1) for k in range(npairs)]
        frames = list(pinned)
        eng.search_pairs(frames, pairs, 16, 4, "sad")
        torch.cuda.synchronize()
        best = 1e9
        for rep in range(3):
            t0 = time.perf_counter()
            eng.search_pairs(frames, pairs, 16, 4, "sad")
            best = min(best, time.perf_counter() - t0)
        print(f"{w}x{h} S4 {npairs} pairs: {best*1e6/npairs:.1f} us/pair", flush=True)
        del eng
