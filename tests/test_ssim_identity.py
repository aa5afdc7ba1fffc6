"""The identity behind the matrix-core SSIM path (csrc/me_ssim.hip,
me_ssim_mfma_kernel), checked on the CPU against the reference's own float
chain.

souravBhat/MotionEstimation src/common/ssim.c:30-42 (computeCrossVar) sums
(ref - Meanref) * (pred - Meanpred) -- int products, the means truncated to
int by the parameter types -- into a float.  For a 16 x 16 block every
product is an int with |product| <= 255^2 and every partial sum has
|sum| <= 256 * 255^2 = 16,646,400 < 2^24, so each float addition is exact:
the chain equals the integer
    cv = sum r c - imc S1r - imr S1c + 256 imr imc,
    sum r c = 127 S1r + 128 S1c - 4161536 - X,  X = sum (127 - c)(r - 128),
whatever the summation order, and X is the i8 GEMM the SSD kernels run.
Here the chain is replayed in float32 in the reference's raster order and
compared with the formula bit for bit on random, flat and extreme blocks.
"""
import numpy as np


def _reference_chain(r, c):
    """computeMean (float sum / 256) truncated to int, then computeCrossVar's
    float32 accumulation in raster order (ssim.c:3-14, 30-42)."""
    mr = np.float32(np.float32(r.sum()) / np.float32(256))
    mc = np.float32(np.float32(c.sum()) / np.float32(256))
    imr, imc = int(mr), int(mc)
    s = np.float32(0)
    for y in range(16):
        for x in range(16):
            s = np.float32(s + np.float32((int(r[y, x]) - imr) * (int(c[y, x]) - imc)))
    return s


def _formula(r, c):
    S1r, S1c = int(r.sum()), int(c.sum())
    imr, imc = S1r >> 8, S1c >> 8
    X = int(((127 - c.astype(np.int64)) * (r.astype(np.int64) - 128)).sum())
    src = 127 * S1r + 128 * S1c - 4161536 - X
    assert src == int((r.astype(np.int64) * c.astype(np.int64)).sum())
    return np.float32(src - imc * S1r - imr * S1c + 256 * imr * imc)


def test_cross_variance_is_an_exact_integer():
    rng = np.random.default_rng(2024)
    cases = []
    for _ in range(300):
        cases.append((rng.integers(0, 256, (16, 16)), rng.integers(0, 256, (16, 16))))
    for v in (0, 1, 127, 128, 254, 255):  # flat blocks
        cases.append((np.full((16, 16), v), rng.integers(0, 256, (16, 16))))
        cases.append((rng.integers(0, 256, (16, 16)), np.full((16, 16), v)))
    for _ in range(40):  # binary 0/255: the largest |products| and partial sums
        cases.append((rng.integers(0, 2, (16, 16)) * 255, rng.integers(0, 2, (16, 16)) * 255))
    cases.append((np.full((16, 16), 255), np.zeros((16, 16), int)))
    cases.append((np.zeros((16, 16), int), np.full((16, 16), 255)))
    for r, c in cases:
        assert _formula(r, c) == _reference_chain(r, c)
