"""A few whole-frame searches of one BASELINE config (diagnostic), for
rocprofv3 kernel-trace / PMC passes:  python tools/dbg/traffic_probe.py 8k sad 3"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import motionestimation_amd as me  # noqa: E402
from motionestimation_amd import synth  # noqa: E402

cfg, cost, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
blk, span = {"1080p": (16, 32), "4k": (16, 64), "8k": (8, 128)}[cfg]
ref, cur = synth.named_pair(cfg)
h, w = ref.shape
nb = me.num_blocks(w, h, blk)
eng = me.Engine(devices=[0])
rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
mv = torch.empty((nb, 2), dtype=torch.int16, device="cuda")
co = torch.empty(nb, dtype=torch.int32, device="cuda")
for _ in range(n):
    eng.full_search_device(rt, ct, blk, span, cost, mv, co)
torch.cuda.synchronize()
eng.close()
