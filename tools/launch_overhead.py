#!/usr/bin/env python3
"""Host-side cost of one me_full_search_device call (ctypes + C ABI + planner
+ launch), measured by issuing N launches of the 1080p search back to back and
timing the host loop (the GPU queue absorbs them)."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import motionestimation_amd as me
from motionestimation_amd import synth
ref, cur = synth.named_pair("1080p")
rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
n = me.num_blocks(1920, 1080, 16)
mv = torch.empty((n, 2), dtype=torch.int16, device="cuda")
co = torch.empty(n, dtype=torch.int32, device="cuda")
eng = me.Engine(devices=[0])
stream = me.engine._current_stream()
for _ in range(5):
    eng.full_search_device(rt, ct, 16, 32, "sad", mv, co, stream=stream)
torch.cuda.synchronize()
N = 200
t0 = time.perf_counter()
for _ in range(N):
    eng.full_search_device(rt, ct, 16, 32, "sad", mv, co, stream=stream)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host issue {1e6*(t1-t0)/N:.1f} us/launch; GPU drain {1e6*(t2-t0)/N:.1f} us/launch")
