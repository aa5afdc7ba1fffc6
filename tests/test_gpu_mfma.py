"""Matrix-core SSD path (i8 MFMA cross term; the S2 term formed per band in
the band-walk kernel on the automatic path (me_band.hip), per workgroup on the
lean path, or read from a prepass plane on the prepass path (me_mfma.hip))
against the oracle and against the VALU kernels, bit-exact (MVs and integer
SSDs).

The MFMA path serves B = 16 SSD on full blocks; tiles of 4x4 blocks, chunks of
L = 45/61 candidate rows, 1-4 groups of 64 candidate columns (S up to 103).
The cases cover every (groups, chunk length) instance, frame edges on all four
sides, tiles with missing block rows / columns, partial right columns and
bottom rows (handed to the VALU kernels), stride != width, stripes whose ref
plane holds only the halo rows, and the extreme key ranges (SSD 0 and the
largest SSD 256 * 255^2)."""
import os

import numpy as np
import pytest

import oracle_lib as O
import motionestimation_amd as me
from motionestimation_amd import synth

pytestmark = pytest.mark.gpu
NT = min(16, os.cpu_count() or 1)


@pytest.fixture(params=["auto", "lean", "prepass"], autouse=True)
def ssd_path(request):
    """Every case on the default matrix-core path (16x16, S <= 64: the
    band-walk kernel), on the lean one (ME_PATH_MFMA_LEAN: S2 per workgroup)
    and on the prepass one (ME_PATH_MFMA_PREPASS: S2 planes); other shapes plan
    as auto.  Cases that switch paths themselves end on auto."""
    me.set_kernel_path(request.param)
    yield request.param
    me.set_kernel_path("auto")


def _pair(rng, h, w, dx=2, dy=-1, noise=3):
    ref = synth._box5(rng.integers(0, 256, (h, w), dtype=np.uint8))
    cur = np.clip(synth.shift_plane(ref, dx, dy).astype(int) + rng.integers(-noise, noise + 1, (h, w)),
                  0, 255).astype(np.uint8)
    return ref, cur


def _check(engine, ref, cur, span, tag, stride=None):
    mv, cost = engine.full_search(ref, cur, 16, span, "ssd", stride=stride)
    omv, ocost, _ = O.full_search(ref, cur, 16, span, "ssd", threads=NT)
    np.testing.assert_array_equal(mv, omv, err_msg=tag)
    np.testing.assert_array_equal(cost, ocost, err_msg=tag)


@pytest.mark.parametrize("span", [1, 2, 3, 7, 8, 13, 16, 17, 24, 31, 32, 40, 47, 48, 63, 64, 80, 103,
                                  104, 128, 150, 192])
def test_mfma_ssd_spans(engine, span):
    """Every (64-column groups, chunk length) instance the planner picks, with
    frame edges on all sides and tiles that lack block rows or columns."""
    rng = np.random.default_rng(1000 + span)
    for (h, w) in [(96, 128), (150, 200), (64, 352)]:
        ref, cur = _pair(rng, h, w, dx=(span % 5) - 2, dy=2 - (span % 3))
        _check(engine, ref, cur, span, f"{h}x{w} S{span}")


def test_mfma_vs_valu_path(engine):
    """Same search on both kernel paths: identical outputs."""
    rng = np.random.default_rng(7)
    try:
        for (h, w, span) in [(288, 352, 16), (200, 320, 32), (176, 240, 64), (120, 176, 7)]:
            ref, cur = _pair(rng, h, w, dx=3, dy=-3)
            me.set_kernel_path("auto")
            a = engine.full_search(ref, cur, 16, span, "ssd")
            me.set_kernel_path("valu")
            b = engine.full_search(ref, cur, 16, span, "ssd")
            np.testing.assert_array_equal(a[0], b[0], err_msg=f"{h}x{w} S{span}")
            np.testing.assert_array_equal(a[1], b[1])
    finally:
        me.set_kernel_path("auto")


def test_mfma_extreme_values(engine):
    """Key range ends: SSD 0 everywhere (all ties), the largest SSD (0 vs 255),
    and mixed saturated planes."""
    h, w = 80, 112
    zeros, full = np.zeros((h, w), np.uint8), np.full((h, w), 255, np.uint8)
    rng = np.random.default_rng(3)
    noise = rng.integers(0, 256, (h, w), dtype=np.uint8)
    binary = (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8)
    for tag, ref, cur in [("flat", full, full), ("zeros", zeros, zeros), ("max", zeros, full),
                          ("max2", full, zeros), ("noise/0", noise, zeros), ("0/noise", zeros, noise),
                          ("binary", binary, np.roll(binary, 3, axis=1)), ("noise", noise, noise)]:
        for span in (5, 32):
            _check(engine, ref, cur, span, f"{tag} S{span}")


@pytest.mark.parametrize("span", [113, 128, 192])
def test_mfma_extreme_values_segmented_bands(engine, span):
    """The block-major kernel splits a band into 16-tile key segments from
    S = 113 on (16 + 2S >= 256 positions): equal costs in two segments must
    resolve to the raster-first (dy, dx).  All-ties and saturated planes on a
    frame wide and tall enough for interior block pairs (40 blocks + 2S)."""
    h, w = 16 * 6 + 2 * span, 16 * 40 + 2 * span
    zeros, full = np.zeros((h, w), np.uint8), np.full((h, w), 255, np.uint8)
    rng = np.random.default_rng(span)
    binary = (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8)
    stripes = np.tile(((np.arange(w) // 2) % 2 * 200 + 20).astype(np.uint8), (h, 1))
    for tag, ref, cur in [("flat", full, full), ("zeros", zeros, zeros), ("max", zeros, full),
                          ("stripes", stripes, np.roll(stripes, 1, axis=1)),
                          ("binary", binary, np.roll(binary, 5, axis=0))]:
        _check(engine, ref, cur, span, f"{tag} S{span} {h}x{w}")


def test_mfma_partial_edges_and_stride(engine):
    """Partial right column / bottom row (VALU kernels beside the MFMA tiles)
    and a row pitch larger than the width."""
    rng = np.random.default_rng(11)
    for (h, w, span) in [(100, 150, 16), (73, 201, 9), (40, 36, 32), (17, 17, 4), (16, 16, 8)]:
        ref, cur = _pair(rng, h, w)
        _check(engine, ref, cur, span, f"{h}x{w} S{span}")
    import torch
    ref, cur = _pair(rng, 96, 160)
    pad_r = np.zeros((96, 200), np.uint8)
    pad_c = np.zeros((96, 200), np.uint8)
    pad_r[:, :160], pad_c[:, :160] = ref, cur
    rt, ct = torch.from_numpy(pad_r).cuda(), torch.from_numpy(pad_c).cuda()
    n = me.num_blocks(160, 96, 16)
    mvt = torch.empty((n, 2), dtype=torch.int16, device="cuda")
    cot = torch.empty(n, dtype=torch.int32, device="cuda")
    engine.full_search_device(rt, ct, 16, 20, "ssd", mvt, cot, width=160, height=96, stride=200)
    torch.cuda.synchronize()
    omv, ocost, _ = O.full_search(ref, cur, 16, 20, "ssd", threads=NT)
    np.testing.assert_array_equal(mvt.cpu().numpy(), omv)
    np.testing.assert_array_equal(cot.cpu().numpy().view(np.uint32), ocost)


def test_mfma_stripes_halo_only(engine):
    """Row stripes whose ref plane holds only [r0*B - S, r1*B + S): the
    prepass and the window DMA see exactly the resident rows."""
    import torch
    rng = np.random.default_rng(5)
    h, w, blk, span = 208, 256, 16, 24
    ref, cur = _pair(rng, h, w, dx=-3, dy=4)
    omv, ocost, _ = O.full_search(ref, cur, blk, span, "ssd", threads=NT)
    nbx = w // blk
    for (r0, r1) in [(0, 3), (3, 7), (7, 13), (5, 6)]:
        y0, y1 = max(0, r0 * blk - span), min(h, r1 * blk + span)
        rt = torch.from_numpy(np.ascontiguousarray(ref[y0:y1])).cuda()
        ct = torch.from_numpy(np.ascontiguousarray(cur[r0 * blk:r1 * blk])).cuda()
        n = (r1 - r0) * nbx
        mvt = torch.empty((n, 2), dtype=torch.int16, device="cuda")
        cot = torch.empty(n, dtype=torch.int32, device="cuda")
        engine.search_stripe_device(rt, y0, ct, r0 * blk, w, h, blk, span, "ssd", r0, r1, mvt, cot)
        torch.cuda.synchronize()
        sl = slice(r0 * nbx, r1 * nbx)
        np.testing.assert_array_equal(mvt.cpu().numpy(), omv[sl], err_msg=f"rows {r0}-{r1}")
        np.testing.assert_array_equal(cot.cpu().numpy().view(np.uint32), ocost[sl])


# ------------------------------------------------------------------ 8x8 blocks
def _check8(engine, ref, cur, span, tag):
    mv, cost = engine.full_search(ref, cur, 8, span, "ssd")
    omv, ocost, _ = O.full_search(ref, cur, 8, span, "ssd", threads=NT)
    np.testing.assert_array_equal(mv, omv, err_msg=tag)
    np.testing.assert_array_equal(cost, ocost, err_msg=tag)


@pytest.mark.parametrize("span", [1, 2, 5, 8, 13, 20, 32, 33, 40, 64, 100, 128])
def test_mfma8_ssd_spans(engine, span):
    """8x8 blocks (one MFMA per output tile): tiles of 4x4 blocks, one to five
    64-column groups per tile (merged across workgroups), partial bottom rows
    and right columns beside the MFMA tiles."""
    rng = np.random.default_rng(2000 + span)
    for (h, w) in [(72, 96), (150, 200), (64, 352), (53, 101)]:
        ref, cur = _pair(rng, h, w, dx=(span % 5) - 2, dy=2 - (span % 3))
        _check8(engine, ref, cur, span, f"B8 {h}x{w} S{span}")


def test_mfma8_vs_valu_and_extremes(engine):
    rng = np.random.default_rng(9)
    try:
        for (h, w, span) in [(288, 352, 16), (200, 320, 48), (160, 240, 128)]:
            ref, cur = _pair(rng, h, w, dx=-3, dy=2)
            me.set_kernel_path("auto")
            a = engine.full_search(ref, cur, 8, span, "ssd")
            me.set_kernel_path("valu")
            b = engine.full_search(ref, cur, 8, span, "ssd")
            np.testing.assert_array_equal(a[0], b[0], err_msg=f"{h}x{w} S{span}")
            np.testing.assert_array_equal(a[1], b[1])
    finally:
        me.set_kernel_path("auto")
    h, w = 64, 104
    zeros, full = np.zeros((h, w), np.uint8), np.full((h, w), 255, np.uint8)
    noise = rng.integers(0, 256, (h, w), dtype=np.uint8)
    for tag, ref, cur in [("flat", full, full), ("max", zeros, full), ("max2", full, zeros),
                          ("noise/0", noise, zeros), ("noise", noise, noise)]:
        _check8(engine, ref, cur, 20, f"B8 {tag}")


@pytest.mark.parametrize("span", [12, 40])
def test_mfma8_stripes_from_partial_reference(engine, span):
    """8x8 SSD stripes whose reference tensor holds only the rows the stripe's
    windows reach (ref_row0 > 0): the search kernel stages the window straight
    from that reference (round 5: no r ^ 0x80 plane), so its row offsets and
    the buffer range at the slice's ends are exercised against the oracle."""
    import torch
    w, h, blk = 328, 236, 8
    rng = np.random.default_rng(77 + span)
    ref, cur = _pair(rng, h, w, dx=5, dy=-4)
    omv, oco, _ = O.full_search(ref, cur, blk, span, "ssd", threads=NT)
    nby, nbx = (h + blk - 1) // blk, w // blk
    omv, oco = omv.reshape(nby, -1, 2), oco.reshape(nby, -1)
    for r0, r1 in [(0, 7), (7, 13), (13, nby - 1), (nby - 1, nby), (3, nby)]:
        y0, y1 = max(r0 * blk - span, 0), min(r1 * blk + span, h)
        ref_t = torch.from_numpy(ref[y0:y1].copy()).cuda()
        cur_t = torch.from_numpy(cur[r0 * blk:min(r1 * blk, h)].copy()).cuda()
        n = (r1 - r0) * omv.shape[1]
        mv = torch.full((n, 2), -9, dtype=torch.int16, device="cuda")
        co = torch.zeros(n, dtype=torch.int32, device="cuda")
        engine.search_stripe_device(ref_t, y0, cur_t, r0 * blk, w, h, blk, span, "ssd", r0, r1, mv, co)
        torch.cuda.synchronize()
        msg = f"S{span} rows {r0}:{r1}"
        np.testing.assert_array_equal(mv.cpu().numpy().reshape(r1 - r0, -1, 2), omv[r0:r1], err_msg=msg)
        np.testing.assert_array_equal(co.cpu().numpy().view(np.uint32).reshape(r1 - r0, -1), oco[r0:r1],
                                      err_msg=msg)
    engine.device_check()


def test_mfma8_8k_s128_sampled(engine):
    """BASELINE configs[4] shape with the reference's cost: 7680x4320, 8x8,
    +-128 SSD on the matrix cores, oracle on sampled block rows."""
    ref, cur = synth.named_pair("8k")
    mv, cost = engine.full_search(ref, cur, 8, 128, "ssd")
    nbx = 960
    for row in (0, 301, 539):
        b0, b1 = row * nbx + 400, row * nbx + 448
        omv, ocost, _ = O.full_search(ref, cur, 8, 128, "ssd", threads=NT, begin=b0, end=b1)
        np.testing.assert_array_equal(mv[b0:b1], omv, err_msg=f"row {row}")
        np.testing.assert_array_equal(cost[b0:b1], ocost)


# ------------------------------------------------------------------ fuzz
def test_mfma_random_shapes(engine):
    """Seeded random frame sizes, ranges and block sizes on every MFMA kernel
    (block-major, 4x4-block tiles, 8x8) and their edge paths, against the
    oracle: widths/heights not multiples of B, ranges from 1 to 192 (B = 16; 79 for B = 8), noise and
    smooth content."""
    rng = np.random.default_rng(4242)
    for it in range(150):
        blk = int(rng.choice([8, 16]))
        span = int(rng.integers(1, 193 if blk == 16 else 80))
        h = int(rng.integers(blk, 200))
        w = int(rng.integers(blk, 260))
        if rng.random() < 0.5:
            ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
            cur = rng.integers(0, 256, (h, w), dtype=np.uint8)
        else:
            ref, cur = _pair(rng, h, w, dx=int(rng.integers(-4, 5)), dy=int(rng.integers(-4, 5)))
        mv, cost = engine.full_search(ref, cur, blk, span, "ssd")
        omv, ocost, _ = O.full_search(ref, cur, blk, span, "ssd", threads=NT)
        tag = f"it{it} {h}x{w} B{blk} S{span}"
        np.testing.assert_array_equal(mv, omv, err_msg=tag)
        np.testing.assert_array_equal(cost, ocost, err_msg=tag)


@pytest.mark.parametrize("span", [72, 128, 192])
def test_mfma_bm_large_ranges_interior_pairs(engine, span):
    """Block-major kernel beyond 16 tiles per band (segmented key index) on a
    frame wide enough for interior block pairs (the mask-free fast path)."""
    rng = np.random.default_rng(3000 + span)
    ref, cur = _pair(rng, 144, 40 * 16 + 2 * span, dx=5, dy=-3)
    _check(engine, ref, cur, span, f"S{span} wide")


def test_mfma_tile_kernel_spans(engine):
    """The 4x4-block-tile kernel (the fallback for rows that are not 16-byte
    aligned), forced through me_set_kernel_path: every (column groups, chunk
    length) instance against the oracle."""
    rng = np.random.default_rng(77)
    try:
        me.set_kernel_path("tiles")
        for span in (1, 7, 16, 17, 32, 47, 48, 64, 80, 103):
            for (h, w) in [(96, 128), (150, 200)]:
                ref, cur = _pair(rng, h, w, dx=(span % 5) - 2, dy=2 - (span % 3))
                _check(engine, ref, cur, span, f"tiles {h}x{w} S{span}")
    finally:
        me.set_kernel_path("auto")


def test_mfma_batch_mixed_alignment(engine):
    """A job table of SSD frames whose planes sit at different byte alignments
    (16, 4, 1 mod 16): the batched matrix-core launch is planned from job 0, so
    misaligned later jobs must send the batch job by job (each on a kernel its
    own alignment allows); every job equals the oracle."""
    import torch
    w, h, blk, span = 320, 192, 16, 16
    frames = [synth.frame_pair(w, h, 60 + f, 3 - f, f - 2) for f in range(4)]
    offs = [0, 4, 1, 16]
    nb = me.num_blocks(w, h, blk)
    plane = w * h
    buf_r = torch.zeros(len(frames) * (plane + 64), dtype=torch.uint8, device="cuda")
    buf_c = torch.zeros_like(buf_r)
    jobs, outs = [], []
    for f, ((r, c), off) in enumerate(zip(frames, offs)):
        base = f * (plane + 64) + off
        rt = buf_r[base:base + plane].view(h, w)
        ct = buf_c[base + (off % 3):base + (off % 3) + plane].view(h, w)
        rt.copy_(torch.from_numpy(r))
        ct.copy_(torch.from_numpy(c))
        mv = torch.full((nb, 2), -9, dtype=torch.int16, device="cuda")
        co = torch.zeros(nb, dtype=torch.int32, device="cuda")
        jobs.append((rt, 0, ct, 0, 0, (h + blk - 1) // blk, mv, co))
        outs.append((mv, co))
    engine.search_stripes_device(w, h, blk, span, "ssd", jobs, stride=w)
    torch.cuda.synchronize()
    engine.device_check()
    for f, ((r, c), (mv, co)) in enumerate(zip(frames, outs)):
        omv, oco, _ = O.full_search(r, c, blk, span, "ssd", threads=NT)
        np.testing.assert_array_equal(mv.cpu().numpy(), omv, err_msg=f"job {f}")
        np.testing.assert_array_equal(co.cpu().numpy().view(np.uint32), oco, err_msg=f"job {f}")


@pytest.mark.parametrize("shape,span", [((720, 1280), 32), ((544, 960), 16), ((368, 656), 64),
                                        ((1080, 1920), 32), ((376, 656), 64), ((1080, 1920), 48)])
def test_band_walk_segments_and_batches(engine, ssd_path, shape, span):
    """The band-walk kernel splits a frame into segments of block rows when
    its strips alone do not fill the CUs (single frames) and walks whole
    strips in batches: one frame, and the same frame in a batch of 6 with
    other frames, against the oracle.  Partial bottom block rows: 1080 =
    67 x 16 + 8 (S 32: searched inside the walk on its own S2 planes; S 48:
    its planes do not fit beside the ring, so a second launch of the lean
    kernel me_mfma_bmv_kernel searches it) and 376 = 23 x 16 + 8 at S 64 (the
    same second launch); 368 = 23 x 16 has none."""
    import torch
    if ssd_path == "prepass":
        pytest.skip("band-walk geometry: the auto and lean paths run the band-walk kernel")
    h, w = shape
    rng = np.random.default_rng(h + span)
    pairs = [_pair(rng, h, w, dx=int(rng.integers(-5, 6)), dy=int(rng.integers(-5, 6))) for _ in range(6)]
    ref, cur = pairs[0]
    _check(engine, ref, cur, span, f"{h}x{w} S{span} single")
    # the auto and lean paths run the band-walk kernel on a single frame too
    # (round 5: a missing scratch check had sent band-walk searches to the
    # VALU kernels, correct but 3x slower)
    engine.full_search(ref, cur, 16, span, "ssd")
    assert me.last_search_path() == "mfma_bandwalk", me.last_search_path()
    dev = torch.device("cuda", 0)
    nb = me.num_blocks(w, h, 16)
    rt = torch.from_numpy(np.stack([r for r, _ in pairs])).to(dev)
    ct = torch.from_numpy(np.stack([c for _, c in pairs])).to(dev)
    mv = torch.empty((6 * nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(6 * nb, dtype=torch.int32, device=dev)
    engine.search_batch_device(rt, 0, ct, 0, w, h, 16, span, "ssd", 0, (h + 15) // 16, mv, co)
    torch.cuda.synchronize()
    assert me.last_search_path() == "mfma_bandwalk", me.last_search_path()
    mv, co = mv.cpu().numpy().reshape(6, nb, 2), co.cpu().numpy().view(np.uint32).reshape(6, nb)
    for f, (r, c) in enumerate(pairs):
        omv, oc, _ = O.full_search(r, c, 16, span, "ssd", threads=NT)
        np.testing.assert_array_equal(mv[f], omv, err_msg=f"frame {f}")
        np.testing.assert_array_equal(co[f], oc, err_msg=f"frame {f}")


@pytest.mark.parametrize("shape,span,frames", [((368, 656), 64, 16), ((360, 640), 32, 32)])
def test_band_walk_xcd_tail_split(engine, ssd_path, shape, span, frames):
    """Batches whose strips fill whole rounds of CUs walk them whole and cut
    each XCD's last partial round into segments (bw_item in me_band.hip):
    368 x 656 S64, 16 frames = 336 strips (42 per XCD: 10 tail strips in 3
    segments each); 360 x 640 S32, 32 frames = 320 strips (8 tail strips in 4
    segments, with the partial bottom row 360 = 22 x 16 + 8)."""
    import torch
    if ssd_path == "prepass":
        pytest.skip("band-walk geometry")
    h, w = shape
    rng = np.random.default_rng(7 * h + span)
    pairs = [_pair(rng, h, w, dx=int(rng.integers(-6, 7)), dy=int(rng.integers(-6, 7))) for _ in range(frames)]
    dev = torch.device("cuda", 0)
    nb = me.num_blocks(w, h, 16)
    rt = torch.from_numpy(np.stack([r for r, _ in pairs])).to(dev)
    ct = torch.from_numpy(np.stack([c for _, c in pairs])).to(dev)
    mv = torch.empty((frames * nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(frames * nb, dtype=torch.int32, device=dev)
    engine.search_batch_device(rt, 0, ct, 0, w, h, 16, span, "ssd", 0, (h + 15) // 16, mv, co)
    torch.cuda.synchronize()
    engine.device_check()
    assert me.last_search_path() == "mfma_bandwalk", me.last_search_path()
    mv, co = mv.cpu().numpy().reshape(frames, nb, 2), co.cpu().numpy().view(np.uint32).reshape(frames, nb)
    for f, (r, c) in enumerate(pairs):
        omv, oc, _ = O.full_search(r, c, 16, span, "ssd", threads=NT)
        np.testing.assert_array_equal(mv[f], omv, err_msg=f"frame {f}")
        np.testing.assert_array_equal(co[f], oc, err_msg=f"frame {f}")


_SEG_SCRIPT = r"""
import sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
import numpy as np
import motionestimation_amd as me
from motionestimation_amd import synth
import oracle_lib as O
assert me._lib.LIB_PATH.endswith("libme_hip_tune.so"), me._lib.LIB_PATH
rng = np.random.default_rng(5)
with me.Engine() as eng:
    for (h, w, span) in [(400, 480, 32), (336, 272, 7), (304, 400, 48)]:
        ref = synth._box5(rng.integers(0, 256, (h, w), dtype=np.uint8))
        cur = synth.shift_plane(ref, 3, -2)
        mv, c = eng.full_search(ref, cur, 16, span, "ssd")
        omv, oc, _ = O.full_search(ref, cur, 16, span, "ssd")
        assert np.array_equal(mv, omv) and np.array_equal(c, oc), (h, w, span)
print("segments ok")
"""


@pytest.mark.parametrize("seg", [1, 2, 3, 5, 7])
def test_band_walk_forced_segment_rows(tmp_path, seg):
    """The tuning build with ME_BW_SEG: segments of 1, 2, 3, 5 and 7 block
    rows (every boundary a prologue re-forms the bands above it), S 7 / 32 / 48."""
    import subprocess
    import sys
    lib = os.path.join(O.REPO, "motionestimation_amd", "lib", "libme_hip_tune.so")
    assert os.path.exists(lib), "build with __graft_entry__.build()"
    script = tmp_path / "seg.py"
    script.write_text(_SEG_SCRIPT.format(repo=O.REPO, tests=os.path.join(O.REPO, "tests")))
    env = dict(os.environ, ME_HIP_LIB="libme_hip_tune.so", ME_BW_SEG=str(seg))
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "segments ok" in r.stdout


@pytest.mark.parametrize("path,want", [("auto", "mfma_bandwalk"), ("prepass", "mfma_prepass"),
                                       ("lean", "mfma_bandwalk"), ("tiles", "mfma_tiles"), ("valu", "valu")])
def test_kernel_path_reported(engine, path, want):
    """me_last_search_path names the kernel family each me_set_kernel_path
    value runs for a 16x16 +-32 SSD search of one small frame (on the
    automatic path the band-walk kernel: its segments run in one round of
    workgroups); SAD runs the VALU kernels on every path."""
    rng = np.random.default_rng(11)
    ref, cur = _pair(rng, 256, 320, dx=2, dy=-1)
    try:
        me.set_kernel_path(path)
        mv, c = engine.full_search(ref, cur, 16, 32, "ssd")
        assert me.last_search_path() == want, (path, me.last_search_path())
        omv, oc, _ = O.full_search(ref, cur, 16, 32, "ssd", threads=NT)
        np.testing.assert_array_equal(mv, omv)
        np.testing.assert_array_equal(c, oc)
        engine.full_search(ref, cur, 16, 32, "sad")
        assert me.last_search_path() == "valu"
    finally:
        me.set_kernel_path("auto")


def test_batched_ssd_partial_right_column_stays_on_mfma(engine, ssd_path):
    """A batch of 16x16 SSD frames whose width is not a multiple of 16 (854 =
    53 x 16 + 6, rows at a 16-byte pitch of 864): launch_mfma_jobs runs it job
    by job (the partial right column goes to the VALU kernels per frame), and
    the context scratch must hold one job's prepass planes for the prepass
    path -- round 5 sized it for the band-walk batch (none) and the fallback
    silently ran every full column on the VALU kernels.  The full
    columns stay on the matrix cores and the fields equal the oracle's."""
    import torch
    h, w, pitch, span, F = 344, 854, 864, 32, 4
    rng = np.random.default_rng(854)
    pairs = [_pair(rng, h, w, dx=int(rng.integers(-4, 5)), dy=int(rng.integers(-4, 5))) for _ in range(F)]
    dev = torch.device("cuda", 0)
    nb = me.num_blocks(w, h, 16)
    pad = lambda a: np.pad(a, ((0, 0), (0, pitch - w)))  # noqa: E731
    rt = torch.from_numpy(np.stack([pad(r) for r, _ in pairs])).to(dev)
    ct = torch.from_numpy(np.stack([pad(c) for _, c in pairs])).to(dev)
    mv = torch.empty((F * nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(F * nb, dtype=torch.int32, device=dev)
    engine.search_batch_device(rt, 0, ct, 0, w, h, 16, span, "ssd", 0, (h + 15) // 16, mv, co)
    torch.cuda.synchronize()
    engine.device_check()
    want = {"auto": "mfma_bandwalk", "lean": "mfma_bandwalk", "prepass": "mfma_prepass"}[ssd_path]
    assert engine.last_search_path() == want, (ssd_path, engine.last_search_path())
    mv, co = mv.cpu().numpy().reshape(F, nb, 2), co.cpu().numpy().view(np.uint32).reshape(F, nb)
    for f, (r, c) in enumerate(pairs):
        omv, oc, _ = O.full_search(r, c, 16, span, "ssd", threads=NT)
        np.testing.assert_array_equal(mv[f], omv, err_msg=f"frame {f}")
        np.testing.assert_array_equal(co[f], oc, err_msg=f"frame {f}")


def test_mfma8_two_tile_workgroups_random_shapes(engine):
    """Round 6: the 8x8 kernel runs two horizontally adjacent 4x4-block tiles
    per workgroup over the union of their candidate columns.  Random widths
    give odd tile counts (the last workgroup's second tile absent), partial
    tiles (nbx % 4 != 0); ranges reach past either
    tile's own columns; every field against the oracle, and the 8x8 MFMA
    kernel must be the one that ran."""
    rng = np.random.default_rng(6262)
    for case in range(12):
        # whole 8x8 blocks (a partial row or column would run the generic
        # kernel after the MFMA one and be the path reported)
        w = 8 * int(rng.integers(5, 45))           # nbx 5 .. 44: tiles_x odd and even
        h = 8 * int(rng.integers(3, 18))
        span = int(rng.choice([3, 9, 16, 31, 47, 64, 100, 128]))
        ref, cur = _pair(rng, h, w, dx=int(rng.integers(-6, 7)), dy=int(rng.integers(-6, 7)))
        tag = f"case {case}: {w}x{h} S{span} tiles_x {((w // 8) + 3) // 4}"
        _check8(engine, ref, cur, span, tag)
        assert engine.last_search_path() == "mfma_8x8", (tag, engine.last_search_path())
