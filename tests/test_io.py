"""File formats (include/me.h §files) on the host: u8 YUV planes
as the reference reads them (src/common/utils.c:29-92) and the MEMV MV-field
file, checked against independent numpy / struct parsing.  No GPU needed."""
import os
import struct

import numpy as np
import pytest

import oracle_lib as O
import motionestimation_amd as me
from motionestimation_amd import io


def test_read_luma_matches_reference_frames(manifest):
    """The committed reference frames (frames/ForemanYF*.yuv, W*H luma bytes)
    read through the library equal the raw bytes."""
    for key in ("ForemanYF1", "ForemanYF2", "ForemanYF4"):
        path = os.path.join(O.GOLDEN, manifest["frames"][key]["file"])
        assert io.yuv_frame_count(path, 352, 288) == 1
        np.testing.assert_array_equal(io.read_luma(path, 352, 288), O.load_frame(key, manifest))


def test_multi_frame_luma_and_i420(tmp_path):
    rng = np.random.default_rng(0)
    w, h, n = 18, 10, 4
    luma = rng.integers(0, 256, (n, h, w), dtype=np.uint8)
    p = tmp_path / "seq.y"
    for i in range(n):
        io.write_yuv(p, luma[i], append=i > 0)
    assert io.yuv_frame_count(p, w, h) == n
    for i in range(n):
        np.testing.assert_array_equal(io.read_luma(p, w, h, i), luma[i])
    # I420: luma then two (w/2 x h/2) chroma planes per frame
    chroma = rng.integers(0, 256, (n, 2 * (h // 2) * (w // 2)), dtype=np.uint8)
    raw = b"".join(luma[i].tobytes() + chroma[i].tobytes() for i in range(n))
    q = tmp_path / "seq.i420"
    q.write_bytes(raw + b"\x01\x02")  # trailing partial frame is not counted
    assert io.yuv_frame_count(q, w, h, "i420") == n
    for i in range(n):
        np.testing.assert_array_equal(io.read_luma(q, w, h, i, "i420"), luma[i])
    # into a strided destination (a column window of a wider plane)
    wide = np.zeros((h, w + 6), np.uint8)
    io.read_luma(p, w, h, 2, out=wide[:, :w])
    np.testing.assert_array_equal(wide[:, :w], luma[2])
    assert not wide[:, w:].any()


def test_yuv_errors(tmp_path):
    p = tmp_path / "short.y"
    p.write_bytes(b"\x00" * 50)
    with pytest.raises(me.MEError) as ei:
        io.read_luma(p, 10, 10)
    assert ei.value.status == me._lib.ME_EIO
    with pytest.raises(me.MEError) as ei:
        io.read_luma(tmp_path / "missing.y", 4, 4)
    assert ei.value.status == me._lib.ME_EIO
    with pytest.raises(me.MEError):
        io.yuv_frame_count(tmp_path / "missing.y", 4, 4)
    with pytest.raises(me.MEError) as ei:
        io.read_luma(p, 0, 4)
    assert ei.value.status == me._lib.ME_EINVAL


def _parse_memv(raw: bytes):
    """Independent reader of the MEMV layout documented in include/me.h."""
    magic, ver, flags, w, h, b, s, cost, n = struct.unpack_from("<4sHHiiiiiI", raw, 0)
    assert magic == b"MEMV" and ver == 1
    nb = ((w + b - 1) // b) * ((h + b - 1) // b)
    off, pairs, mvs, costs = 32, [], [], []
    for _ in range(n):
        pairs.append(struct.unpack_from("<ii", raw, off))
        off += 8
        mvs.append(np.frombuffer(raw, "<i2", 2 * nb, off).reshape(nb, 2))
        off += 4 * nb
        if flags & 1:
            costs.append(np.frombuffer(raw, "<u4", nb, off))
            off += 4 * nb
    assert off == len(raw)
    return (w, h, b, s, cost, flags), pairs, np.array(mvs), (np.array(costs) if flags & 1 else None)


def test_memv_round_trip_and_layout(tmp_path):
    rng = np.random.default_rng(1)
    w, h, blk, span = 100, 75, 16, 9
    nb = me.num_blocks(w, h, blk)
    mv = rng.integers(-span, span + 1, (3, nb, 2)).astype(np.int16)
    cost = rng.integers(0, 1 << 20, (3, nb)).astype(np.uint32)
    pairs = [(0, 1), (0, 2), (5, 7)]
    p = tmp_path / "f.memv"
    io.write_mv(p, w, h, blk, span, "sad", mv, cost, pairs=pairs)
    hdr, pr, mv2, c2 = io.read_mv(p)
    assert (hdr["width"], hdr["height"], hdr["block_size"], hdr["search_range"]) == (w, h, blk, span)
    assert hdr["cost"] == me.ME_COST_SAD and hdr["has_cost"] and hdr["n_pairs"] == 3
    assert pr.tolist() == [list(x) for x in pairs]
    np.testing.assert_array_equal(mv2, mv)
    np.testing.assert_array_equal(c2, cost)
    geo, pp, mv3, c3 = _parse_memv(p.read_bytes())
    assert geo == (w, h, blk, span, me.ME_COST_SAD, 1)
    assert pp == pairs
    np.testing.assert_array_equal(mv3, mv)
    np.testing.assert_array_equal(c3, cost)


def test_memv_defaults_without_cost(tmp_path):
    w, h, blk = 64, 48, 8
    nb = me.num_blocks(w, h, blk)
    mv = np.arange(2 * nb, dtype=np.int16).reshape(nb, 2)  # one pair, 2-D form
    p = tmp_path / "g.memv"
    io.write_mv(p, w, h, blk, 4, "ssd", mv)
    hdr, pr, mv2, c2 = io.read_mv(p)
    assert not hdr["has_cost"] and c2 is None
    assert pr.tolist() == [[0, 1]]
    np.testing.assert_array_equal(mv2[0], mv)
    assert os.path.getsize(p) == 32 + 8 + 4 * nb


def test_memv_rejects_damage(tmp_path):
    w, h, blk = 32, 32, 8
    nb = me.num_blocks(w, h, blk)
    p = tmp_path / "d.memv"
    io.write_mv(p, w, h, blk, 4, "ssd", np.zeros((2, nb, 2), np.int16), np.zeros((2, nb), np.uint32))
    raw = p.read_bytes()
    (tmp_path / "trunc.memv").write_bytes(raw[:-1])
    (tmp_path / "long.memv").write_bytes(raw + b"\x00")
    (tmp_path / "magic.memv").write_bytes(b"XXXX" + raw[4:])
    for name in ("trunc", "long", "magic"):
        with pytest.raises(me.MEError) as ei:
            io.read_mv(tmp_path / f"{name}.memv")
        assert ei.value.status == me._lib.ME_EIO, name
    with pytest.raises(me.MEError) as ei:  # shape mismatch caught before writing
        io.write_mv(p, w, h, blk, 4, "ssd", np.zeros((nb + 1, 2), np.int16))
    assert ei.value.status == me._lib.ME_EINVAL
