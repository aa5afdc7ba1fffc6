"""Extended seeded fuzz of the HIP path against the oracle (more cases than
tests/test_gpu_fuzz.py, same generators): SAD / SSD at B = 8 and 16 and
random sizes, spans and contents, plus SSIM on smaller shapes.  Prints one
line per failure and a summary; exit status 1 on any mismatch.
usage: python3 tools/dbg/fuzz_more.py [cases] [seed] [aligned]
(aligned: widths a multiple of 16, so the matrix-core SSD / SSIM paths run)"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle_lib as O  # noqa: E402
import motionestimation_amd as me  # noqa: E402
from test_gpu_fuzz import _frames  # noqa: E402

cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 9090
aligned = len(sys.argv) > 3 and sys.argv[3] == "aligned"
rng = np.random.default_rng(seed)
eng = me.Engine(devices=[0])
bad = 0
paths = {}
for k in range(cases):
    cost = str(rng.choice(["sad", "ssd", "ssd", "ssim"]))
    blk = int(rng.choice([8, 16, 16] if cost != "ssim" else [8, 16]))
    wmax, hmax = (400, 300) if cost != "ssim" else (200, 150)
    w, h = int(rng.integers(max(blk, 24), wmax)), int(rng.integers(max(blk, 24), hmax))
    if aligned:
        w = max(16, w // 16 * 16)
    span = int(rng.integers(0 if not aligned else 1, 130 if cost != "ssim" else 70))
    kind = str(rng.choice(["smooth", "smooth", "noise", "flat", "binary"]))
    ref, cur = _frames(rng, w, h, kind)
    mv, c = eng.full_search(ref, cur, blk, span, cost)
    ocost = "mse" if cost == "ssd" else cost
    omv, oc, _ = O.full_search(ref, cur, blk, span, ocost, threads=16)
    ok = np.array_equal(mv, omv) and np.array_equal(c, oc)
    pth = eng.last_search_path()
    paths[pth] = paths.get(pth, 0) + 1
    if not ok:
        bad += 1
        print(f"MISMATCH case {k}: {w}x{h} B{blk} S{span} {kind} {cost} path {eng.last_search_path()}",
              flush=True)
    elif k % 25 == 0:
        print(f"case {k} ok ({w}x{h} B{blk} S{span} {kind} {cost}, {eng.last_search_path()})", flush=True)
eng.close()
print(f"{cases} cases, {bad} mismatches; last kernel family per case: {paths}", flush=True)
sys.exit(1 if bad else 0)
