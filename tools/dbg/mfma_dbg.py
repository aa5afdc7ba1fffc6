import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import oracle_lib as O
import motionestimation_amd as me
from test_gpu_mfma import _pair
eng = me.Engine()
for span, shape in [(3, (96, 128)), (4, (96, 128)), (5, (96, 128)), (7, (64, 64))]:
    rng = np.random.default_rng(1000 + span)
    h, w = shape
    ref, cur = _pair(rng, h, w, dx=(span % 5) - 2, dy=2 - (span % 3))
    mv, cost = eng.full_search(ref, cur, 16, span, "ssd")
    omv, ocost, _ = O.full_search(ref, cur, 16, span, "ssd", threads=8)
    bad = np.nonzero((mv != omv).any(1) | (cost != ocost))[0]
    print("span", span, shape, "bad blocks", len(bad))
    for b in bad[:12]:
        print("  blk", b, "(bx,by)", b % (w // 16), b // (w // 16), "got", mv[b], cost[b], "want", omv[b], ocost[b])
