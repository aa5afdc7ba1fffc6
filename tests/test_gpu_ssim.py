"""SSIM cost (ME_COST_SSIM) on the GPU, bit-exact with the
reference's CPU SSIM search (src/common/ssim.c:3-108): score bits on every
block, MVs wherever the best score is > 0 (elsewhere the reference's MV is
uninitialised and this build defines (0, 0))."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
import motionestimation_amd as me
from motionestimation_amd import synth

pytestmark = pytest.mark.gpu


def _check(mv, bits, gmv, gscore, name):
    np.testing.assert_array_equal(bits, gscore.view(np.uint32), err_msg=name)
    pos = gscore > 0
    np.testing.assert_array_equal(mv[pos].astype(np.int32), gmv[pos], err_msg=name)
    assert (mv[~pos] == 0).all(), name


def test_ssim_reference_goldens(engine, manifest):
    """Every SSIM golden from the unmodified reference, incl. full-size 1080p."""
    for c in manifest["ssim_cases"]:
        cur, ref = O.load_frame(c["cur"], manifest), O.load_frame(c["ref"], manifest)
        gmv, gscore = O.load_case(c)
        mv, bits = engine.full_search(ref, cur, c["blk"], c["span"], "ssim")
        _check(mv, bits, gmv, gscore, c["name"])


@pytest.mark.parametrize("blk,span,shape", [(16, 5, (75, 100)), (8, 9, (64, 72)),
                                            (32, 3, (96, 96)), (4, 6, (30, 41)),
                                            (16, 120, (150, 160))])
def test_ssim_vs_oracle_shapes(engine, blk, span, shape):
    """Partial blocks, w*h > 256 (float chains that round), and a window too
    large for LDS (S = 120: read from global memory)."""
    h, w = shape
    ref, cur = synth.frame_pair(w, h, blk * 7 + span, 2, -1)
    mv, bits = engine.full_search(ref, cur, blk, span, "ssim")
    omv, obits, oscore = O.full_search(ref, cur, blk, span, "ssim")
    np.testing.assert_array_equal(bits, obits)
    np.testing.assert_array_equal(mv, omv)


def test_ssim_through_stripes_pairs_and_device_lists(engine):
    """The same kernel behind the stripe, pair-streaming and multi-device paths."""
    seq = synth.sequence(160, 112, 3, 9, 2, 1)
    omv = [O.full_search(seq[k], seq[k + 1], 16, 7, "ssim") for k in range(2)]
    mv, c = engine.search_pairs(list(seq), [(0, 1), (1, 2)], 16, 7, "ssim")
    for k in range(2):
        np.testing.assert_array_equal(mv[k], omv[k][0])
        np.testing.assert_array_equal(c[k], omv[k][1])
    with me.Engine(devices=[0, 0, 0]) as eng:
        mv3, c3 = eng.full_search(seq[0], seq[1], 16, 7, "ssim")
    np.testing.assert_array_equal(mv3, omv[0][0])
    np.testing.assert_array_equal(c3, omv[0][1])


def test_ssim_c_driver_matches_reference_driver(tmp_path, manifest):
    """bin/mes_hip --cost ssim: the reference SSIM driver's score line and its
    5-plane output file, byte for byte (src/cpu/main_ssim.c)."""
    exe = os.path.join(O.REPO, "bin", "mes_hip")
    assert os.path.exists(exe), "build with __graft_entry__.build()"
    for d in manifest["ssim_driver"]:
        cur = os.path.join(O.GOLDEN, manifest["frames"][d["cur"]]["file"])
        ref = os.path.join(O.GOLDEN, manifest["frames"][d["ref"]]["file"])
        r = subprocess.run([exe, cur, ref, str(tmp_path), str(d["blk"]), str(d["span"]), "352",
                            "288", "--cost", "ssim"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert d["score_line"] in r.stdout, r.stdout
        out = (tmp_path / f"output_{d['blk']}_{d['span']}.yuv").read_bytes()
        assert hashlib.sha256(out).hexdigest() == d["output_sha256"]


def test_ssim_reference_interface(engine, manifest):
    """find_best_blks(cost='ssim') / find_best_blk_ssim mirror main_ssim.c:15-29."""
    f1, f2 = O.load_frame("ForemanYF1", manifest), O.load_frame("ForemanYF2", manifest)
    c = [c for c in manifest["ssim_cases"] if c["name"] == "ssim_foreman21_b16_s7"][0]
    gmv, gscore = O.load_case(c)
    pf = me.create_prediction_frame(f2, 352, 288, 16)
    scores = me.find_best_blks(pf, f1, 7, cost="ssim", engine=engine)
    np.testing.assert_array_equal(scores.view(np.uint32), gscore.view(np.uint32))
    np.testing.assert_array_equal(me.reference_api.mv_field(pf).astype(np.int32), gmv)
    blk = pf.blks[57]
    s = me.find_best_blk_ssim(pf, f1, blk, 7, engine=engine)
    assert np.float32(s).view(np.uint32) == gscore.view(np.uint32)[57]
    assert [blk.motion_vectorX, blk.motion_vectorY] == gmv[57].tolist()


@pytest.mark.parametrize("span", [0, 3, 16, 33, 64])
def test_ssim_partial_bottom_row_every_height(engine, span):
    """16 x 16 blocks: the full-width blocks of a partial bottom row (H % 16 =
    1 .. 15; N = 16 (H % 16) pixels, powers of two and not) run on the matrix
    cores from their own 16 x (H % 16) statistics plane; smooth, flat and
    binary frames, a partial right column beside them."""
    rng = np.random.default_rng(600 + span)
    for hbh in range(1, 16):
        h, w = 16 * 3 + hbh, 16 * 5 + (hbh % 3) * 5
        kind = ("smooth", "flat", "binary")[hbh % 3]
        if kind == "smooth":
            ref, cur = synth.frame_pair(w, h, hbh + span, 2, -1)
        elif kind == "flat":
            ref = np.full((h, w), 97, np.uint8)
            ref[::3] = 98
            cur = np.full((h, w), 97, np.uint8)
            cur[:, ::5] = 40
        else:
            ref = (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8)
            cur = (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8)
        mv, bits = engine.full_search(ref, cur, 16, span, "ssim")
        omv, obits, _ = O.full_search(ref, cur, 16, span, "ssim")
        what = f"{w}x{h} S{span} {kind}"
        np.testing.assert_array_equal(bits, obits, err_msg=what)
        np.testing.assert_array_equal(mv, omv, err_msg=what)


def test_ssim_partial_bottom_row_alone_on_a_device():
    """A device list that leaves one device only the partial bottom row (and
    one a run of full rows ending at it): each launch builds the planes it needs."""
    ref, cur = synth.frame_pair(200, 16 * 4 + 12, 31, 3, 2)
    omv, obits, _ = O.full_search(ref, cur, 16, 20, "ssim")
    for devs in ([0, 0, 0, 0, 0], [0, 0]):
        with me.Engine(devices=devs) as eng:
            mv, bits = eng.full_search(ref, cur, 16, 20, "ssim")
        np.testing.assert_array_equal(bits, obits, err_msg=str(devs))
        np.testing.assert_array_equal(mv, omv, err_msg=str(devs))
