"""Frame-pair streaming (me_search_pairs) on the GPU: every pair
bit-identical to the reference goldens / the oracle, whatever the pair list,
frame memory (pageable, pinned, strided) or device list."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
import motionestimation_amd as me
from motionestimation_amd import synth

pytestmark = pytest.mark.gpu


def _case(manifest, name):
    return [c for c in manifest["cases"] if c["name"] == name][0]


def test_multi_reference_foreman_goldens(engine, manifest):
    """frames/ForemanYF{1,2,4}: 1->2, 1->4 and 4->1 in one call, each pair equal
    to the unmodified reference's dump (main.c:144-158 run once per pair)."""
    frames = [O.load_frame(k, manifest) for k in ("ForemanYF1", "ForemanYF2", "ForemanYF4")]
    pairs = [(0, 1), (0, 2), (2, 0)]
    names = ["foreman21_b8_s12", "foreman41_b8_s12", "foreman14_b8_s12"]
    mv, cost = engine.search_pairs(frames, pairs, 8, 12, "ssd")
    assert mv.shape == (3, me.num_blocks(352, 288, 8), 2)
    for i, name in enumerate(names):
        gmv, _ = O.load_case(_case(manifest, name))
        np.testing.assert_array_equal(mv[i].astype(np.int32), gmv, err_msg=name)
        ref, cur = frames[pairs[i][0]], frames[pairs[i][1]]
        _, ossd, _ = O.full_search(ref, cur, 8, 12, "mse")
        np.testing.assert_array_equal(cost[i], ossd, err_msg=name)


@pytest.mark.parametrize("cost", ["sad", "ssd"])
def test_sequence_pageable_and_pinned(engine, cost):
    """A 7-frame pan, consecutive pairs: pageable frames (staged) and frames in
    me_host_alloc memory (direct DMA) give the oracle's result on every pair."""
    w, h, n = 320, 240, 7
    seq = synth.sequence(w, h, n, 11, 3, -2)
    pairs = [(k, k + 1) for k in range(n - 1)]
    mv, c = engine.search_pairs(list(seq), pairs, 16, 16, cost)
    pinned = me.pinned_frames(n, h, w)
    pinned[:] = seq
    mvp, cp = engine.search_pairs(list(pinned), pairs, 16, 16, cost)
    np.testing.assert_array_equal(mvp, mv)
    np.testing.assert_array_equal(cp, c)
    for k, (r, q) in enumerate(pairs):
        omv, oc, _ = O.full_search(seq[r], seq[q], 16, 16, cost)
        np.testing.assert_array_equal(mv[k], omv, err_msg=f"pair {k}")
        np.testing.assert_array_equal(c[k], oc, err_msg=f"pair {k}")
    # the pan is recovered: interior blocks point at (-3, +2)
    assert (mv[:, 40:60] == np.array([-3, 2], np.int16)).all(axis=-1).mean() > 0.8


def test_pair_lists_and_reuse(engine):
    """Odd pair lists: repeated pairs, (f, f), a frame reused after a gap,
    backwards pairs; then a different frame size on the same context."""
    seq = synth.sequence(96, 80, 5, 3, 2, 1)
    pairs = [(0, 1), (1, 1), (4, 0), (0, 1), (2, 3), (3, 2), (0, 4)]
    mv, c = engine.search_pairs(list(seq), pairs, 8, 7, "sad")
    for k, (r, q) in enumerate(pairs):
        omv, oc, _ = O.full_search(seq[r], seq[q], 8, 7, "sad")
        np.testing.assert_array_equal(mv[k], omv, err_msg=f"pair {k}")
        np.testing.assert_array_equal(c[k], oc, err_msg=f"pair {k}")
    assert not mv[1].any() and not c[1].any()  # (f, f): zero vectors, zero cost
    seq2 = synth.sequence(100, 75, 3, 4, -1, 3)  # partial blocks, new slot size
    mv2, c2 = engine.search_pairs(list(seq2), [(0, 1), (1, 2)], 16, 9, "ssd")
    for k, (r, q) in enumerate([(0, 1), (1, 2)]):
        omv, oc, _ = O.full_search(seq2[r], seq2[q], 16, 9, "ssd")
        np.testing.assert_array_equal(mv2[k], omv)
        np.testing.assert_array_equal(c2[k], oc)


def test_strided_frames_through_c_abi(engine):
    """Frames with row pitch > width (views into wider planes), pinned and
    pageable, through the raw C entry point."""
    w, h, pitch, n = 128, 96, 160, 3
    seq = synth.sequence(w, h, n, 5, -2, 1)
    pinned = me.pinned_frames(n, h, pitch)
    pageable = np.zeros((n, h, pitch), np.uint8)
    pinned[:, :, :w] = seq
    pageable[:, :, :w] = seq
    pinned[:, :, w:] = 255
    pageable[:, :, w:] = 255
    pairs = np.array([[0, 1], [1, 2], [2, 0]], np.int32)
    nb = me.num_blocks(w, h, 8)
    for buf in (pinned, pageable):
        ptrs = (ctypes.c_void_p * n)(*[buf[k].ctypes.data for k in range(n)])
        mv = np.zeros((3, nb, 2), np.int16)
        cost = np.zeros((3, nb), np.uint32)
        me._lib.check(me._lib.lib().me_search_pairs(
            engine._h, ptrs, n, w, h, pitch, 8, 10, me.ME_COST_SAD, pairs.ctypes.data, 3,
            mv.ctypes.data, cost.ctypes.data), engine._h)
        for k, (r, q) in enumerate(pairs):
            omv, oc, _ = O.full_search(seq[r], seq[q], 8, 10, "sad")
            np.testing.assert_array_equal(mv[k], omv)
            np.testing.assert_array_equal(cost[k], oc)


def test_pairs_split_across_device_list():
    """Contexts over [0, 0] and [0, 0, 0]: contiguous runs of pairs driven by
    one host thread each, results identical to the single-device context."""
    seq = synth.sequence(192, 128, 9, 8, 1, 1)
    pairs = [(k, k + 1) for k in range(8)] + [(0, 8)]
    with me.Engine() as one:
        mv1, c1 = one.search_pairs(list(seq), pairs, 16, 12, "sad")
    for devs in ([0, 0], [0, 0, 0]):
        with me.Engine(devices=devs) as eng:
            mv, c = eng.search_pairs(list(seq), pairs, 16, 12, "sad")
            np.testing.assert_array_equal(mv, mv1)
            np.testing.assert_array_equal(c, c1)
    omv, oc, _ = O.full_search(seq[0], seq[8], 16, 12, "sad")
    np.testing.assert_array_equal(mv1[-1], omv)
    np.testing.assert_array_equal(c1[-1], oc)


def test_pair_errors(engine):
    seq = synth.sequence(32, 32, 2, 1, 0, 0)
    for pairs in ([(0, 2)], [(-1, 0)]):
        with pytest.raises(me.MEError) as ei:
            engine.search_pairs(list(seq), pairs, 8, 4, "sad")
        assert ei.value.status == me._lib.ME_EINVAL
    with pytest.raises(me.MEError) as ei:
        engine.search_pairs(list(seq), [(0, 1)], 0, 4, "sad")
    assert ei.value.status == me._lib.ME_EINVAL
    mv, c = engine.search_pairs(list(seq), np.zeros((0, 2), np.int32), 8, 4, "sad")
    assert mv.shape[0] == 0 and c.shape[0] == 0


def test_seq_driver_foreman_i420(tmp_path, manifest):
    """bin/mes_seq on an I420 file of Foreman YF1, YF2, YF4 with --ref first:
    the MEMV file holds the reference's 1->2 and 1->4 fields."""
    import os
    import subprocess
    exe = os.path.join(O.REPO, "bin", "mes_seq")
    assert os.path.exists(exe), "build with __graft_entry__.build()"
    frames = [O.load_frame(k, manifest) for k in ("ForemanYF1", "ForemanYF2", "ForemanYF4")]
    chroma = np.full(2 * 176 * 144, 128, np.uint8)
    seq = tmp_path / "foreman.i420"
    seq.write_bytes(b"".join(f.tobytes() + chroma.tobytes() for f in frames))
    out = tmp_path / "f.memv"
    r = subprocess.run([exe, str(seq), "352", "288", "8", "12", "--layout", "i420", "--ref",
                        "first", "--repeat", "3", "--mv", str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Computation time:" in r.stdout
    hdr, pairs, mv, cost = me.io.read_mv(out)
    assert pairs.tolist() == [[0, 1], [0, 2]] and hdr["has_cost"]
    for k, name in enumerate(["foreman21_b8_s12", "foreman41_b8_s12"]):
        gmv, _ = O.load_case(_case(manifest, name))
        np.testing.assert_array_equal(mv[k].astype(np.int32), gmv, err_msg=name)


def _long_pair_list(n_frames):
    """> 16 batches of the 1, 2, 3, 4, 6, 8 ramp: consecutive pairs, (f, f)
    pairs, backwards pairs and frame 0 reused after a long gap (its slot was
    freed and reused meanwhile), so the batch-event ring and the record bounce
    regions wrap and slots are reused after their last reader's event slot was
    overwritten."""
    pairs = []
    for k in range(n_frames - 1):
        pairs.append((k, k + 1))
        if k % 7 == 3:
            pairs.append((k, k))
        if k % 11 == 5:
            pairs.append((k + 1, k - 2))
    pairs.append((0, n_frames - 1))
    pairs.append((n_frames - 1, 0))
    return pairs


def _check_pairs(seq, pairs, mv, c, blk, rng, cost):
    for k, (r, q) in enumerate(pairs):
        omv, oc, _ = O.full_search(seq[r], seq[q], blk, rng, cost, threads=1)
        np.testing.assert_array_equal(mv[k], omv, err_msg=f"pair {k} ({r}, {q})")
        np.testing.assert_array_equal(c[k], oc, err_msg=f"pair {k} ({r}, {q})")


@pytest.mark.parametrize("pinned", [False, True])
def test_long_pair_list_ring_wrap(engine, pinned):
    """>= 150 small pairs (> 16 batches): every record against the oracle, from
    pageable and from me_host_alloc frames (the event ring, the
    bounce-region ring, the drain bound and slot reuse had no result check)."""
    w, h, n = 64, 48, 130
    seq = synth.sequence(w, h, n, 21, 1, -1)
    pairs = _long_pair_list(n)
    assert len(pairs) >= 150
    frames = list(seq)
    if pinned:
        buf = me.pinned_frames(n, h, w)
        buf[:] = seq
        frames = list(buf)
    mv, c = engine.search_pairs(frames, pairs, 8, 7, "sad")
    _check_pairs(seq, pairs, mv, c, 8, 7, "sad")
    # and again on the same context (slots, events and bounce regions reused)
    mv2, c2 = engine.search_pairs(frames, pairs[::-1], 8, 7, "sad")
    np.testing.assert_array_equal(mv2[::-1], mv)
    np.testing.assert_array_equal(c2[::-1], c)


_TUNE_SCRIPT = r"""
import sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
import numpy as np
import motionestimation_amd as me
from motionestimation_amd import synth
import oracle_lib as O
from test_gpu_stream import _long_pair_list, _check_pairs
assert me._lib.LIB_PATH.endswith("libme_hip_tune.so"), me._lib.LIB_PATH
w, h, n = 64, 48, 130
seq = synth.sequence(w, h, n, 21, 1, -1)
pairs = _long_pair_list(n)
with me.Engine() as eng:
    for pinned in (False, True):
        frames = list(seq)
        if pinned:
            buf = me.pinned_frames(n, h, w); buf[:] = seq; frames = list(buf)
        mv, c = eng.search_pairs(frames, pairs, 8, 7, "ssd")
        _check_pairs(seq, pairs, mv, c, 8, 7, "ssd")
print("tuned pipeline ok", len(pairs))
"""


def test_long_pair_list_unbounded_ahead_fixed_batches(tmp_path):
    """The tuning build with ME_STREAM_AHEAD=9 (host unbounded ahead of the
    GPU) and ME_STREAM_RAMP=0 (fixed 8-pair batches): the same long pair list,
    SSD, pinned and pageable, every pair against the oracle."""
    import os
    import subprocess
    import sys
    lib = os.path.join(O.REPO, "motionestimation_amd", "lib", "libme_hip_tune.so")
    assert os.path.exists(lib), "build with __graft_entry__.build()"
    script = tmp_path / "tuned.py"
    script.write_text(_TUNE_SCRIPT.format(repo=O.REPO, tests=os.path.join(O.REPO, "tests")))
    env = dict(os.environ, ME_HIP_LIB="libme_hip_tune.so", ME_STREAM_AHEAD="9", ME_STREAM_RAMP="0")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "tuned pipeline ok" in r.stdout
