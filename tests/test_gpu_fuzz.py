"""Seeded random configurations through the C ABI against the oracle
(oracle/me_oracle.c, the restatement of src/cpu/main.c:18-82), bit for bit.

Each case draws a frame size (odd widths and heights included, so partial
right columns and bottom rows occur), a block size, a search range (0 .. 70:
S mod 4 = 0 takes the SAD kernels' fold, other S the unfolded groups), a
content kind (smooth shifted pairs, noise, all-ties flat frames, 0/255 binary
frames) and a cost, so every kernel family the planner picks for small frames
is exercised: the generic kernel, the item kernel at B = 8 / 16, the MFMA SSD
kernels, and the float replay of SSD for blocks with w*h > 256.

SSD is compared with the oracle's float-MSE mode (the reference's own
argmin, main.c:18-64): the MV field must equal it and the reported cost is the
integer SSD of that vector.  SSIM (the reference's CPU SSIM search,
src/common/ssim.c:3-108) is compared score bit for score bit on smaller
random shapes."""
import os

import numpy as np
import pytest

import oracle_lib as O
from motionestimation_amd import synth

pytestmark = pytest.mark.gpu
NT = min(16, os.cpu_count() or 1)


def _frames(rng, w, h, kind):
    if kind == "flat":
        v = np.full((h, w), int(rng.integers(0, 256)), np.uint8)
        return v, v.copy()
    if kind == "noise":
        return (rng.integers(0, 256, (h, w), dtype=np.uint8),
                rng.integers(0, 256, (h, w), dtype=np.uint8))
    if kind == "binary":
        return ((rng.integers(0, 2, (h, w)) * 255).astype(np.uint8),
                (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8))
    return synth.frame_pair(w, h, int(rng.integers(1, 1 << 30)), int(rng.integers(-9, 10)),
                            int(rng.integers(-9, 10)))


@pytest.mark.parametrize("seed", range(6))
def test_random_configs_against_oracle(engine, seed):
    rng = np.random.default_rng(4242 + seed)
    for case in range(20):
        blk = int(rng.choice([4, 7, 8, 12, 16, 24, 32]))
        # about 64..320 pixels a side, never smaller than one block
        w = int(rng.integers(max(blk, 40), 321))
        h = int(rng.integers(max(blk, 40), 241))
        span = int(rng.integers(0, 71))
        kind = str(rng.choice(["smooth", "smooth", "noise", "flat", "binary"]))
        cost = str(rng.choice(["sad", "ssd"]))
        ref, cur = _frames(rng, w, h, kind)
        mv, c = engine.full_search(ref, cur, blk, span, cost)
        omv, oc, _ = O.full_search(ref, cur, blk, span, "mse" if cost == "ssd" else "sad",
                                   threads=NT)
        what = f"seed {seed} case {case}: {w}x{h} B{blk} S{span} {kind} {cost}"
        np.testing.assert_array_equal(mv, omv, err_msg=what)
        np.testing.assert_array_equal(c, oc, err_msg=what)


@pytest.mark.parametrize("seed", range(2))
def test_random_ssim_configs_against_oracle(engine, seed):
    """The SSIM cost (float replay of src/common/ssim.c) on random shapes:
    full blocks read the patch-statistics plane, partial ones compute their own;
    score bits and MVs equal the oracle's."""
    rng = np.random.default_rng(777 + seed)
    for case in range(10):
        blk = int(rng.choice([4, 8, 12, 16, 24]))
        w = int(rng.integers(max(blk, 24), 161))
        h = int(rng.integers(max(blk, 24), 121))
        span = int(rng.integers(0, 25))
        kind = str(rng.choice(["smooth", "smooth", "noise", "flat", "binary"]))
        ref, cur = _frames(rng, w, h, kind)
        mv, bits = engine.full_search(ref, cur, blk, span, "ssim")
        omv, obits, _ = O.full_search(ref, cur, blk, span, "ssim", threads=NT)
        what = f"seed {seed} case {case}: {w}x{h} B{blk} S{span} {kind} ssim"
        np.testing.assert_array_equal(bits, obits, err_msg=what)
        np.testing.assert_array_equal(mv, omv, err_msg=what)
