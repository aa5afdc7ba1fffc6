"""GPU parity: the HIP path through the C ABI against the reference goldens
and the oracle, bit-exact (integer MVs and costs; the reference's float MSE
score reproduced bit for bit)."""
import os

import numpy as np
import pytest

import oracle_lib as O
import motionestimation_amd as me
from motionestimation_amd import synth

pytestmark = pytest.mark.gpu
NT = min(16, os.cpu_count() or 1)


def _mse_bits(cost, blk, w, h):
    """(float)SSD / (float)(bw*bh) per block, as the reference rounds it."""
    nbx, nby = (w + blk - 1) // blk, (h + blk - 1) // blk
    bw = np.minimum(blk, w - np.arange(nbx) * blk)
    bh = np.minimum(blk, h - np.arange(nby) * blk)
    area = (bh[:, None] * bw[None, :]).reshape(-1).astype(np.float32)
    return (cost.astype(np.float32) / area).view(np.uint32)


def test_golden_cases_ssd(engine, manifest):
    """Every golden case from the unmodified reference: same MVs; MSE bits."""
    for c in manifest["cases"]:
        if c["width"] > 2000:
            continue
        cur, ref = O.load_frame(c["cur"], manifest), O.load_frame(c["ref"], manifest)
        gmv, gmse = O.load_case(c)
        mv, cost = engine.full_search(ref, cur, c["blk"], c["span"], "ssd")
        np.testing.assert_array_equal(mv.astype(np.int32), gmv, err_msg=c["name"])
        if c["blk"] <= 16:
            np.testing.assert_array_equal(_mse_bits(cost, c["blk"], c["width"], c["height"]),
                                          gmse.view(np.uint32), err_msg=c["name"])
        # cost = integer SSD of the reference's chosen vector
        _, ossd, _ = O.full_search(ref, cur, c["blk"], c["span"], "mse", threads=NT)
        np.testing.assert_array_equal(cost, ossd, err_msg=c["name"])


def test_golden_cases_sad(engine, manifest):
    for c in manifest["cases"]:
        if c["width"] > 2000:
            continue
        cur, ref = O.load_frame(c["cur"], manifest), O.load_frame(c["ref"], manifest)
        mv, cost = engine.full_search(ref, cur, c["blk"], c["span"], "sad")
        omv, ocost, _ = O.full_search(ref, cur, c["blk"], c["span"], "sad", threads=NT)
        np.testing.assert_array_equal(mv, omv, err_msg=c["name"])
        np.testing.assert_array_equal(cost, ocost, err_msg=c["name"])


@pytest.mark.parametrize("blk", [8, 16])
@pytest.mark.parametrize("span", [0, 1, 2, 3, 5, 7, 16, 32, 33])
def test_fast_sad_kernel_shapes(engine, blk, span):
    """qsad kernel across dx alignments (S mod 4), chunk padding, partial
    bottom rows (H % B != 0) and a partial right column (W % B != 0)."""
    rng = np.random.default_rng(blk * 100 + span)
    for (h, w) in [(72, 96), (75, 100), (40, 200)]:
        ref = synth._box5(rng.integers(0, 256, (h, w), dtype=np.uint8))
        cur = np.clip(synth.shift_plane(ref, 2, -1).astype(int) + rng.integers(-3, 4, (h, w)), 0,
                      255).astype(np.uint8)
        mv, cost = engine.full_search(ref, cur, blk, span, "sad")
        omv, ocost, _ = O.full_search(ref, cur, blk, span, "sad", threads=NT)
        np.testing.assert_array_equal(mv, omv, err_msg=f"{h}x{w} B{blk} S{span}")
        np.testing.assert_array_equal(cost, ocost)


def test_ties_flat_frame_sad(engine):
    """Flat frames: all candidates tie; the raster-first one must win."""
    ref = np.full((64, 96), 77, np.uint8)
    for blk, span in [(16, 32), (8, 13), (16, 7)]:
        mv, cost = engine.full_search(ref, ref, blk, span, "sad")
        omv, ocost, _ = O.full_search(ref, ref, blk, span, "sad")
        np.testing.assert_array_equal(mv, omv)
        assert (cost == 0).all()


def test_stride_and_device_api(engine):
    import torch
    rng = np.random.default_rng(3)
    h, w, blk, span = 96, 130, 16, 9
    big_ref = rng.integers(0, 256, (h, w + 6), dtype=np.uint8)
    big_cur = rng.integers(0, 256, (h, w + 6), dtype=np.uint8)
    ref, cur = big_ref[:, :w].copy(), big_cur[:, :w].copy()
    omv, ocost, _ = O.full_search(ref, cur, blk, span, "sad")
    # host API with a padded pitch
    mv, cost = engine.full_search(big_ref, big_cur, blk, span, "sad")  # full width first
    n = me.num_blocks(w, h, blk)
    L = me._lib.lib()
    mv2 = np.zeros((n, 2), np.int16)
    c2 = np.zeros(n, np.uint32)
    me._lib.check(L.me_full_search(engine._h, big_ref.ctypes.data, big_cur.ctypes.data, w, h,
                                   w + 6, blk, span, 1, mv2.ctypes.data, c2.ctypes.data),
                  engine._h)
    np.testing.assert_array_equal(mv2, omv)
    np.testing.assert_array_equal(c2, ocost)
    # device API on HBM-resident tensors
    rt = torch.from_numpy(ref).cuda()
    ct = torch.from_numpy(cur).cuda()
    mvt = torch.zeros((n, 2), dtype=torch.int16, device="cuda")
    cot = torch.zeros(n, dtype=torch.int32, device="cuda")
    engine.full_search_device(rt, ct, blk, span, "sad", mvt, cot)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(mvt.cpu().numpy(), omv)
    np.testing.assert_array_equal(cot.cpu().numpy().view(np.uint32), ocost)


def test_stripe_device_api_halo_only(engine):
    """Each stripe sees only its cur rows + S-row ref halo (device pointers
    offset to the stripe origin); concatenated stripes == full frame."""
    import torch
    from motionestimation_amd import shard
    ref, cur = synth.frame_pair(640, 360, 11, 4, -2)
    for blk, span, cost, world in [(16, 32, "sad", 3), (8, 12, "ssd", 4), (16, 7, "sad", 5)]:
        omv, ocost, _ = O.full_search(ref, cur, blk, span, cost, threads=NT)
        mvs, costs = [], []
        for st in shard.plan(640, 360, blk, span, world):
            rt = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).cuda()
            ct = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).cuda()
            n = max(st.nblocks, 1)
            mvt = torch.zeros((n, 2), dtype=torch.int16, device="cuda")
            cot = torch.zeros(n, dtype=torch.int32, device="cuda")
            if st.nblocks:
                engine.search_stripe_device(rt, st.ref_y0, ct, st.cur_y0, 640, 360, blk, span, cost,
                                            st.row_begin, st.row_end, mvt, cot)
            torch.cuda.synchronize()
            mvs.append(mvt.cpu().numpy()[:st.nblocks])
            costs.append(cot.cpu().numpy().view(np.uint32)[:st.nblocks])
        np.testing.assert_array_equal(np.concatenate(mvs), omv)
        np.testing.assert_array_equal(np.concatenate(costs), ocost)


def test_multi_shard_context_on_one_gpu():
    """A context over device ids [0, 0, 0]: stripes + gather inside the library."""
    ref, cur = synth.frame_pair(320, 240, 5, -3, 2)
    with me.Engine(devices=[0, 0, 0]) as eng:
        for cost in ("sad", "ssd"):
            mv, c = eng.full_search(ref, cur, 16, 16, cost)
            omv, oc, _ = O.full_search(ref, cur, 16, 16, cost)
            np.testing.assert_array_equal(mv, omv)
            np.testing.assert_array_equal(c, oc)


def test_reference_adapter_and_interface(engine, manifest):
    """create_prediction_frame / find_best_blks / output planes as the reference
    driver uses them; the published output_4_{7,15}.yuv and PSNR reproduce."""
    f1, f4 = O.load_frame("ForemanYF1", manifest), O.load_frame("ForemanYF4", manifest)
    for key, info in manifest["published"].items():
        pf = me.create_prediction_frame(f4, 352, 288, info["blk"])
        me.find_best_blks(pf, f1, info["span"], engine=engine)
        planes, psnr = me.output_planes(pf, f1, engine=engine)
        pub = np.fromfile(os.path.join(O.GOLDEN, info["file"]), np.uint8).reshape(5 * 288, 352)
        np.testing.assert_array_equal(planes, pub, err_msg=key)
    pf = me.create_prediction_frame(f4, 352, 288, 8)
    scores = me.find_best_blks(pf, f1, 12, engine=engine)
    _, psnr = me.output_planes(pf, f1, engine=engine)
    assert "%.6f" % psnr == "31.816000"
    g = [c for c in manifest["cases"] if c["name"] == "foreman41_b8_s12"][0]
    _, gmse = O.load_case(g)
    np.testing.assert_array_equal(scores.view(np.uint32), gmse.view(np.uint32))


def test_c_adapter_fills_reference_block_records(engine, manifest):
    import ctypes
    f1, f2 = O.load_frame("ForemanYF1", manifest), O.load_frame("ForemanYF2", manifest)
    n = me.num_blocks(352, 288, 16)

    class Blk(ctypes.Structure):
        _fields_ = [(f, ctypes.c_int) for f in (
            "idx_x", "idx_y", "top_left_x", "top_left_y", "bottom_right_x", "bottom_right_y",
            "width", "height", "is_best_match_found", "motion_vectorX", "motion_vectorY")]

    assert ctypes.sizeof(Blk) == 44
    blks = (Blk * n)()
    r32, c32 = f1.astype(np.int32), f2.astype(np.int32)
    me._lib.check(me._lib.lib().me_find_best_blocks(engine._h, r32.ctypes.data, c32.ctypes.data,
                                                     352, 288, 16, 16, blks, n), engine._h)
    g = [c for c in manifest["cases"] if c["name"] == "foreman21_b16_s16"][0]
    gmv, _ = O.load_case(g)
    got = np.array([[b.motion_vectorX, b.motion_vectorY] for b in blks])
    np.testing.assert_array_equal(got, gmv)
    assert all(b.is_best_match_found == 1 for b in blks)
    # planes that did not come from 8-bit samples are refused, not truncated
    for bad in (256, -1, 1 << 20):
        r_bad = r32.copy()
        r_bad[100, 200] = bad
        st = me._lib.lib().me_find_best_blocks(engine._h, r_bad.ctypes.data, c32.ctypes.data,
                                               352, 288, 16, 16, blks, n)
        assert st == me._lib.ME_EINVAL, bad
        assert b"outside [0, 255]" in me._lib.lib().me_last_error(engine._h)
        c_bad = c32.copy()
        c_bad[0, 0] = bad
        assert me._lib.lib().me_find_best_blocks(engine._h, r32.ctypes.data, c_bad.ctypes.data,
                                                 352, 288, 16, 16, blks, n) == me._lib.ME_EINVAL


def test_error_paths(engine):
    ref = np.zeros((32, 32), np.uint8)
    for blk, span in [(0, 4), (65, 4), (8, -1), (8, 5000)]:
        with pytest.raises(me.MEError) as ei:
            engine.full_search(ref, ref, blk, span, "sad")
        assert ei.value.status == me._lib.ME_EINVAL
    with pytest.raises(me.MEError):
        engine.full_search(ref, ref, 8, 4, "nope")
    # planes of 2 GiB or more are refused before any device work
    st = me._lib.lib().me_full_search(engine._h, ref.ctypes.data, ref.ctypes.data, 32, 32,
                                      1 << 26, 8, 4, me.ME_COST_SAD,
                                      np.zeros(64, np.int16).ctypes.data, None)
    assert st == me._lib.ME_EUNSUPPORTED


@pytest.mark.slow
def test_full_1080p_both_costs(engine, manifest):
    """BASELINE configs[2] at full size: SSD vs the reference golden, SAD vs oracle."""
    c = [c for c in manifest["cases"] if c["name"] == "synth1080p_b16_s32"][0]
    ref, cur = synth.named_pair("1080p")
    gmv, gmse = O.load_case(c)
    mv, cost = engine.full_search(ref, cur, 16, 32, "ssd")
    np.testing.assert_array_equal(mv.astype(np.int32), gmv)
    np.testing.assert_array_equal(_mse_bits(cost, 16, 1920, 1080), gmse.view(np.uint32))
    mv, cost = engine.full_search(ref, cur, 16, 32, "sad")
    omv, ocost, _ = O.full_search(ref, cur, 16, 32, "sad", threads=NT)
    np.testing.assert_array_equal(mv, omv)
    np.testing.assert_array_equal(cost, ocost)


@pytest.mark.slow
def test_full_4k_ssd_golden_and_sad_properties(engine, manifest):
    """BASELINE configs[3]: SSD vs the reference golden (full frame); SAD vs the
    oracle on sampled block rows (top, middle, bottom)."""
    c = [c for c in manifest["cases"] if c["name"] == "synth4k_b16_s64"][0]
    ref, cur = synth.named_pair("4k")
    gmv, gmse = O.load_case(c)
    mv, cost = engine.full_search(ref, cur, 16, 64, "ssd")
    np.testing.assert_array_equal(mv.astype(np.int32), gmv)
    np.testing.assert_array_equal(_mse_bits(cost, 16, 3840, 2160), gmse.view(np.uint32))
    mv, cost = engine.full_search(ref, cur, 16, 64, "sad")
    nbx = 240
    for row in (0, 67, 134):
        omv, ocost, _ = O.full_search(ref, cur, 16, 64, "sad", threads=NT, begin=row * nbx,
                                      end=(row + 1) * nbx)
        np.testing.assert_array_equal(mv[row * nbx:(row + 1) * nbx], omv)
        np.testing.assert_array_equal(cost[row * nbx:(row + 1) * nbx], ocost)


@pytest.mark.slow
def test_8k_b8_s128_sampled(engine):
    """BASELINE configs[4] (8x8, +-128, 7680x4320): full GPU frame, oracle on
    sampled block rows; SAD lower-bounded by the zero-vector... property:
    cost <= SAD at the true shift for interior blocks."""
    ref, cur = synth.named_pair("8k")
    mv, cost = engine.full_search(ref, cur, 8, 128, "sad")
    nbx = 960
    for row in (0, 270, 539):
        omv, ocost, _ = O.full_search(ref, cur, 8, 128, "sad", threads=NT, begin=row * nbx,
                                      end=row * nbx + 96)
        np.testing.assert_array_equal(mv[row * nbx:row * nbx + 96], omv)
        np.testing.assert_array_equal(cost[row * nbx:row * nbx + 96], ocost)
    # property over the whole frame: the chosen cost never exceeds the SAD of
    # the generator's true displacement (cur = ref shifted by (+40, -27)).
    r = ref.astype(np.int32)
    c = cur.astype(np.int32)
    nby = 540
    for by in range(2, nby - 6, 97):
        for bx in range(6, nbx - 6, 131):
            y, x = by * 8, bx * 8
            true_sad = np.abs(c[y:y + 8, x:x + 8] - r[y + 27:y + 35, x - 40:x - 32]).sum()
            assert cost[by * nbx + bx] <= true_sad


def test_c_driver_reproduces_published_output(tmp_path, manifest):
    """bin/mes_hip (C host driver on the ABI, reference argv) writes the
    reference's published output_4_{7,15}.yuv byte for byte."""
    import subprocess
    exe = os.path.join(O.REPO, "bin", "mes_hip")
    assert os.path.exists(exe), "build with __graft_entry__.build()"
    f1 = os.path.join(O.GOLDEN, manifest["frames"]["ForemanYF1"]["file"])
    f4 = os.path.join(O.GOLDEN, manifest["frames"]["ForemanYF4"]["file"])
    for key, info in manifest["published"].items():
        r = subprocess.run([exe, f4, f1, str(tmp_path), "4", str(info["span"]), "352", "288",
                            "--mv", str(tmp_path / "mv.bin")], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        out = (tmp_path / f"output_4_{info['span']}.yuv").read_bytes()
        pub = open(os.path.join(O.GOLDEN, info["file"]), "rb").read()
        assert out == pub, key
        assert "Computation time:" in r.stdout
        hdr, pairs, mv, cost = me.io.read_mv(tmp_path / "mv.bin")
        assert (hdr["block_size"], hdr["search_range"], hdr["n_pairs"]) == (4, info["span"], 1)
        gmv, _ = O.load_case([c for c in manifest["cases"]
                              if c["name"] == f"foreman41_b4_s{info['span']}"][0])
        np.testing.assert_array_equal(mv[0].astype(np.int32), gmv)
    r = subprocess.run([exe, f4, f1, str(tmp_path), "8", "12", "352", "288"], capture_output=True,
                       text=True, timeout=120)
    assert "PSNR: 31.816000" in r.stdout


def test_flow_kernel_full_frames(engine):
    """The barrier-free SAD kernel (me_flow_kernel: 1080p-class frames, S = 32,
    >= 2 tiles per CU) against the oracle: all-ties flat frames, noise, the
    h = 8 bottom row, an odd block-row count, and a padded row pitch; S = 16
    (the item kernel) beside it."""
    import torch
    rng = np.random.default_rng(77)
    cases = [(1088, 1920, 32, "flat"), (1080, 1920, 32, "noise"), (1080, 1920, 16, "smooth"),
             (1040, 2048, 32, "smooth")]
    for h, w, span, kind in cases:
        if kind == "flat":
            ref = cur = np.full((h, w), 91, np.uint8)
        elif kind == "noise":
            ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
            cur = rng.integers(0, 256, (h, w), dtype=np.uint8)
        else:
            ref, cur = synth.frame_pair(w, h, 5, -6, 4)
        mv, cost = engine.full_search(ref, cur, 16, span, "sad")
        omv, ocost, _ = O.full_search(ref, cur, 16, span, "sad", threads=NT)
        np.testing.assert_array_equal(mv, omv, err_msg=f"{h}x{w} S{span} {kind}")
        np.testing.assert_array_equal(cost, ocost, err_msg=f"{h}x{w} S{span} {kind}")
    # padded pitch (16-byte multiple) on the device API
    ref, cur = synth.frame_pair(1920, 1080, 9, 2, -5)
    pr, pc = np.zeros((1080, 1984), np.uint8), np.zeros((1080, 1984), np.uint8)
    pr[:, :1920], pc[:, :1920] = ref, cur
    n = me.num_blocks(1920, 1080, 16)
    mvt = torch.empty((n, 2), dtype=torch.int16, device="cuda")
    cot = torch.empty(n, dtype=torch.int32, device="cuda")
    engine.full_search_device(torch.from_numpy(pr).cuda(), torch.from_numpy(pc).cuda(), 16, 32,
                              "sad", mvt, cot, width=1920, height=1080, stride=1984)
    torch.cuda.synchronize()
    omv, ocost, _ = O.full_search(ref, cur, 16, 32, "sad", threads=NT)
    np.testing.assert_array_equal(mvt.cpu().numpy(), omv)
    np.testing.assert_array_equal(cot.cpu().numpy().view(np.uint32), ocost)


@pytest.mark.parametrize("span", [16, 32])
def test_stripes_of_multi_gpu_splits(engine, span):
    """Every stripe of 3-, 4- and 8-way 1080p splits (the per-rank unit of the
    multi-GPU search: the persistent item kernel on small stripes, the flow
    kernel on large ones), a width with a partial last flow tile (121
    blocks), an all-ties frame, and frames too small to give every CU work;
    each stripe searched twice (the kernels' counters reset themselves)."""
    import torch
    from motionestimation_amd import shard
    rng = np.random.default_rng(span)
    frames = [(1920, 1080, "smooth"), (1936, 1080, "noise"), (1920, 1088, "flat"),
              (352, 288, "smooth"), (96, 64, "noise"), (48, 48, "smooth")]
    for w, h, kind in frames:
        if kind == "flat":
            ref = cur = np.full((h, w), 13, np.uint8)
        elif kind == "noise":
            ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
            cur = rng.integers(0, 256, (h, w), dtype=np.uint8)
        else:
            ref, cur = synth.frame_pair(w, h, 21, 3, -5)
        omv, ocost, _ = O.full_search(ref, cur, 16, span, "sad", threads=NT)
        worlds = (1, 3, 4, 8) if h >= 1080 else (1, 2)
        for world in worlds:
            for st in shard.plan(w, h, 16, span, world):
                if not st.nblocks:
                    continue
                rt = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).cuda()
                ct = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).cuda()
                mvt = torch.full((st.nblocks, 2), -9, dtype=torch.int16, device="cuda")
                cot = torch.zeros(st.nblocks, dtype=torch.int32, device="cuda")
                for _ in range(2):  # twice: the merge buffers reset themselves
                    engine.search_stripe_device(rt, st.ref_y0, ct, st.cur_y0, w, h, 16, span,
                                                "sad", st.row_begin, st.row_end, mvt, cot)
                torch.cuda.synchronize()
                b0, b1 = st.row_begin * st.nbx, st.row_end * st.nbx
                msg = f"{w}x{h} {kind} S{span} {world}-way rows {st.row_begin}:{st.row_end}"
                np.testing.assert_array_equal(mvt.cpu().numpy(), omv[b0:b1], err_msg=msg)
                np.testing.assert_array_equal(cot.cpu().numpy().view(np.uint32), ocost[b0:b1],
                                              err_msg=msg)
    engine.device_check()


@pytest.mark.parametrize("cost,blk,span,w,h,ways", [
    ("sad", 16, 32, 1920, 1080, 8),   # flow kernel, one launch for the batch (h = 8 bottom row)
    ("sad", 16, 32, 1920, 1080, 1),   # whole frames batched
    ("sad", 16, 16, 1000, 700, 3),    # item kernel over the batch; generic kernel for the
                                      # partial right column and the h = 12 bottom row
    ("ssd", 16, 32, 1920, 1080, 4),   # matrix cores, frame by frame
    ("sad", 8, 24, 640, 360, 2),      # 8x8 item kernel, one launch for the batch
])
def test_batch_search_equals_per_frame(engine, cost, blk, span, w, h, ways):
    """me_full_search_batch_device: F stripes (or whole frames) of different
    frames in one call equal the oracle frame by frame, with records laid out
    frame-major; padded frame strides are honoured."""
    import torch
    from motionestimation_amd import shard
    F = 3
    base_ref, base_cur = synth.frame_pair(w, h, 31, 4, -3)
    frames = [(np.roll(base_ref, 37 * f, axis=1), np.roll(base_cur, 37 * f, axis=1))
              for f in range(F)]
    oracle = [O.full_search(r, c, blk, span, cost, threads=NT)[:2] for r, c in frames]
    for st in shard.plan(w, h, blk, span, ways):
        if not st.nblocks:
            continue
        pad = 48  # frames further apart than their rows: strides are taken as given
        rr, cr = st.ref_y1 - st.ref_y0, st.cur_y1 - st.cur_y0
        ref_b = torch.zeros((F, rr + pad, w), dtype=torch.uint8, device="cuda")
        cur_b = torch.zeros((F, cr + pad, w), dtype=torch.uint8, device="cuda")
        for f, (r, c) in enumerate(frames):
            ref_b[f, :rr] = torch.from_numpy(r[st.ref_y0:st.ref_y1].copy())
            cur_b[f, :cr] = torch.from_numpy(c[st.cur_y0:st.cur_y1].copy())
        mv = torch.full((F * st.nblocks, 2), -5, dtype=torch.int16, device="cuda")
        co = torch.zeros(F * st.nblocks, dtype=torch.int32, device="cuda")
        for _ in range(2):
            engine.search_batch_device(ref_b, st.ref_y0, cur_b, st.cur_y0, w, h, blk, span, cost,
                                       st.row_begin, st.row_end, mv, co)
        torch.cuda.synchronize()
        mv, co = mv.cpu().numpy(), co.cpu().numpy().view(np.uint32)
        b0, b1 = st.row_begin * st.nbx, st.row_end * st.nbx
        for f in range(F):
            n = st.nblocks
            msg = f"{cost} {w}x{h} B{blk} S{span} rows {st.row_begin}:{st.row_end} frame {f}"
            np.testing.assert_array_equal(mv[f * n:(f + 1) * n], oracle[f][0][b0:b1], err_msg=msg)
            np.testing.assert_array_equal(co[f * n:(f + 1) * n], oracle[f][1][b0:b1], err_msg=msg)
    engine.device_check()


@pytest.mark.parametrize("cost", ["ssd", "sad"])
def test_batch_past_one_launch(engine, cost):
    """A batch longer than one launch's job table (MAX_JOBS = 32): 40 frames
    of a frame with a partial bottom block row run as 32 + 8 jobs (SSD: shared
    prepass + block-major launches; SAD: the flow kernel's job table) and equal
    the oracle frame by frame."""
    import torch
    F, w, h, blk, span = 40, 160, 120, 16, 32
    base_ref, base_cur = synth.frame_pair(w, h, 7, -2, 5)
    frames = [(np.roll(base_ref, 11 * f, axis=1), np.roll(base_cur, 11 * f, axis=1))
              for f in range(F)]
    ref_b = torch.from_numpy(np.stack([r for r, _ in frames])).cuda()
    cur_b = torch.from_numpy(np.stack([c for _, c in frames])).cuda()
    nb = me.num_blocks(w, h, blk)
    mv = torch.full((F * nb, 2), -5, dtype=torch.int16, device="cuda")
    co = torch.zeros(F * nb, dtype=torch.int32, device="cuda")
    engine.search_batch_device(ref_b, 0, cur_b, 0, w, h, blk, span, cost, 0, (h + blk - 1) // blk,
                               mv, co)
    torch.cuda.synchronize()
    mv, co = mv.cpu().numpy(), co.cpu().numpy().view(np.uint32)
    for f, (r, c) in enumerate(frames):
        omv, oco, _ = O.full_search(r, c, blk, span, cost, threads=NT)
        np.testing.assert_array_equal(mv[f * nb:(f + 1) * nb], omv, err_msg=f"{cost} frame {f}")
        np.testing.assert_array_equal(co[f * nb:(f + 1) * nb], oco, err_msg=f"{cost} frame {f}")
    engine.device_check()


def test_batch_search_argument_checks(engine):
    import torch
    L = me._lib.lib()
    ref = torch.zeros((2, 64, 64), dtype=torch.uint8, device="cuda")
    mv = torch.zeros((2 * 16, 2), dtype=torch.int16, device="cuda")
    base = dict(ref_stride=64 * 64, cur_stride=64 * 64, n=2)

    def call(ref_stride=base["ref_stride"], cur_stride=base["cur_stride"], n=base["n"]):
        return L.me_full_search_batch_device(engine._h, ref.data_ptr(), ref_stride, 0,
                                             ref.data_ptr(), cur_stride, 0, 64, 64, 64, 16, 8,
                                             1, 0, 4, n, mv.data_ptr(), None, None)
    assert call() == me._lib.ME_OK
    assert call(ref_stride=64 * 63) == me._lib.ME_EINVAL   # frames would overlap
    assert call(cur_stride=100) == me._lib.ME_EINVAL
    assert call(n=0) == me._lib.ME_EINVAL
    assert call(ref_stride=1 << 31) == me._lib.ME_EUNSUPPORTED
    torch.cuda.synchronize()


@pytest.mark.parametrize("cost,blk,span,w,h,ways", [
    ("sad", 16, 32, 1920, 1080, 8),   # flow kernel: one launch for stripes of different rows
    ("sad", 16, 32, 1920, 1080, 4),
    ("sad", 16, 16, 1000, 700, 3),    # item kernel over the jobs + generic leftovers
    ("ssd", 16, 32, 1920, 1080, 8),   # matrix cores, job by job
])
def test_stripe_jobs_of_different_rows(engine, cost, blk, span, w, h, ways):
    """me_search_stripes_device with bench.py's rotated step: job f is stripe
    (r + f) % N of frame f, so one call mixes top, interior and bottom stripes
    of different heights; every job equals the oracle on its rows."""
    import torch
    from motionestimation_amd import shard
    F = max(ways, 3)
    base_ref, base_cur = synth.frame_pair(w, h, 41, -5, 2)
    frames = [(np.roll(base_ref, 37 * f, axis=1), np.roll(base_cur, 37 * f, axis=1))
              for f in range(F)]
    plan = shard.plan(w, h, blk, span, ways)
    for r in (0, ways - 1):
        jobs, want = [], []
        for f in range(F):
            st = plan[(r + f) % ways]
            if not st.nblocks:
                continue
            rt = torch.from_numpy(frames[f][0][st.ref_y0:st.ref_y1].copy()).cuda()
            ct = torch.from_numpy(frames[f][1][st.cur_y0:st.cur_y1].copy()).cuda()
            mv = torch.full((st.nblocks, 2), -3, dtype=torch.int16, device="cuda")
            co = torch.zeros(st.nblocks, dtype=torch.int32, device="cuda")
            jobs.append((rt, st.ref_y0, ct, st.cur_y0, st.row_begin, st.row_end, mv, co))
            want.append((f, st))
        for _ in range(2):
            engine.search_stripes_device(w, h, blk, span, cost, jobs)
        torch.cuda.synchronize()
        for (f, st), job in zip(want, jobs):
            omv, oco, _ = O.full_search(*frames[f], blk, span, cost, threads=NT,
                                        begin=st.row_begin * st.nbx, end=st.row_end * st.nbx)
            msg = f"{cost} {w}x{h} rank {r} frame {f} rows {st.row_begin}:{st.row_end}"
            np.testing.assert_array_equal(job[6].cpu().numpy(), omv, err_msg=msg)
            np.testing.assert_array_equal(job[7].cpu().numpy().view(np.uint32), oco, err_msg=msg)
    engine.device_check()


@pytest.mark.parametrize("cfg,blk,span,ways,F", [
    ("4k", 16, 64, 8, 8),   # bench.py's 4K 8-way step: one item-kernel launch, pitch-272 instance
    ("4k", 16, 64, 1, 3),   # whole 4K frames batched (dynamic tile pulls over the batch)
    ("8k", 8, 128, 2, 2),   # 8x8 strip walk per job (>= 32 tiles wide and 32 rows tall)
])
def test_item_kernel_jobs_equal_single_searches(engine, cfg, blk, span, ways, F):
    """The item kernel over a job table (me_search_stripes_device with bench.py's
    rotated step: job f = stripe (r + f) % N of frame f) equals one
    me_full_search_device per frame on the same rows, bit for bit; the
    single-frame searches are pinned by the full-frame hashes
    (tests/test_gpu_fullframe.py)."""
    import torch
    from motionestimation_amd import shard
    base_ref, base_cur = synth.named_pair(cfg)
    h, w = base_ref.shape
    nb = me.num_blocks(w, h, blk)
    frames = [(np.roll(base_ref, 37 * f, axis=1), np.roll(base_cur, 37 * f, axis=1))
              for f in range(F)]
    want = []
    for r, c in frames:
        rt, ct = torch.from_numpy(r).cuda(), torch.from_numpy(c).cuda()
        mv = torch.empty((nb, 2), dtype=torch.int16, device="cuda")
        co = torch.empty(nb, dtype=torch.int32, device="cuda")
        engine.full_search_device(rt, ct, blk, span, "sad", mv, co)
        torch.cuda.synchronize()
        want.append((mv.cpu().numpy(), co.cpu().numpy()))
        del rt, ct
    plan = shard.plan(w, h, blk, span, ways)
    for rank in sorted({0, ways - 1}):
        own = [plan[(rank + f) % ways] for f in range(F)]
        jobs, keep = [], []
        for f, st in enumerate(own):
            r, c = frames[f]
            rt = torch.from_numpy(r[st.ref_y0:st.ref_y1].copy()).cuda()
            ct = torch.from_numpy(c[st.cur_y0:st.cur_y1].copy()).cuda()
            mv = torch.full((st.nblocks, 2), -7, dtype=torch.int16, device="cuda")
            co = torch.zeros(st.nblocks, dtype=torch.int32, device="cuda")
            jobs.append((rt, st.ref_y0, ct, st.cur_y0, st.row_begin, st.row_end, mv, co))
            keep.append((st, mv, co))
        engine.search_stripes_device(w, h, blk, span, "sad", jobs)
        torch.cuda.synchronize()
        for f, (st, mv, co) in enumerate(keep):
            b0, b1 = st.row_begin * st.nbx, st.row_end * st.nbx
            msg = f"{cfg} {ways}-way rank {rank} frame {f} rows {st.row_begin}:{st.row_end}"
            np.testing.assert_array_equal(mv.cpu().numpy(), want[f][0][b0:b1], err_msg=msg)
            np.testing.assert_array_equal(co.cpu().numpy(), want[f][1][b0:b1], err_msg=msg)
        del jobs, keep
    engine.device_check()


def test_random_job_tables_equal_per_job_searches(engine):
    """Property: me_search_stripes_device over a random job table (random row
    ranges of random frames, empty jobs, more jobs than one launch holds)
    equals one me_full_search_stripe_device call per job, for every kernel
    family the shapes reach (flow, item, generic, matrix cores)."""
    import torch
    rng = np.random.default_rng(2024)
    shapes = [  # cost, B, S, W, H
        ("sad", 16, 32, 1920, 1080),   # flow kernel
        ("sad", 16, 16, 1000, 700),    # item kernel + generic leftovers
        ("sad", 8, 24, 640, 360),      # 8x8 item kernel
        ("ssd", 16, 32, 640, 480),     # matrix cores, job by job
        ("ssd", 8, 12, 330, 203),      # 8x8 matrix cores + partial column and row
        ("sad", 12, 9, 400, 300),      # generic kernel only
    ]
    for cost, blk, span, w, h in shapes:
        nby = (h + blk - 1) // blk
        nbx = (w + blk - 1) // blk
        n = int(rng.integers(2, 21))
        pairs = [synth.frame_pair(w, h, int(rng.integers(1, 1 << 30)), int(rng.integers(-6, 7)),
                                  int(rng.integers(-6, 7))) for _ in range(min(n, 4))]
        jobs, singles = [], []
        for j in range(n):
            r, c = pairs[j % len(pairs)]
            r0 = int(rng.integers(0, nby))
            r1 = r0 if j == 1 else int(rng.integers(r0 + 1, nby + 1))  # job 1 empty
            y0, y1 = max(r0 * blk - span, 0), min(r1 * blk + span, h)
            ref_t = torch.from_numpy(r[y0:y1].copy()).cuda() if y1 > y0 else torch.zeros(
                (1, w), dtype=torch.uint8, device="cuda")
            cur_t = torch.from_numpy(c[r0 * blk:min(r1 * blk, h)].copy()).cuda() if r1 > r0 else \
                torch.zeros((1, w), dtype=torch.uint8, device="cuda")
            nblk = (r1 - r0) * nbx
            mv = torch.full((max(nblk, 1), 2), -9, dtype=torch.int16, device="cuda")
            co = torch.zeros(max(nblk, 1), dtype=torch.int32, device="cuda")
            jobs.append((ref_t, y0, cur_t, r0 * blk, r0, r1, mv, co))
            mv1, co1 = mv.clone(), co.clone()
            if r1 > r0:
                engine.search_stripe_device(ref_t, y0, cur_t, r0 * blk, w, h, blk, span, cost,
                                            r0, r1, mv1, co1)
            singles.append((mv1, co1))
        engine.search_stripes_device(w, h, blk, span, cost, jobs)
        torch.cuda.synchronize()
        for j, ((_, _, _, _, r0, r1, mv, co), (mv1, co1)) in enumerate(zip(jobs, singles)):
            msg = f"{cost} B{blk} S{span} {w}x{h} job {j}/{n} rows {r0}:{r1}"
            np.testing.assert_array_equal(mv.cpu().numpy(), mv1.cpu().numpy(), err_msg=msg)
            np.testing.assert_array_equal(co.cpu().numpy(), co1.cpu().numpy(), err_msg=msg)
    engine.device_check()
