"""File formats over libme_hip.so (include/me.h).

u8 YUV planes (the reference's yuvReadFrame / yuvWriteFrame,
src/common/utils.c:29-92, without its int32 widening) and the MV-field file
(``MEMV``: 32-byte header, then per pair the raster-order (mvx, mvy) int16
records and optional u32 costs).  Errors raise :class:`MEError`.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib
from ._lib import ME_YUV_I420, ME_YUV_LUMA, MEError, check
from .engine import cost_code, num_blocks

_LAYOUT = {"luma": ME_YUV_LUMA, "y": ME_YUV_LUMA, "i420": ME_YUV_I420,
           ME_YUV_LUMA: ME_YUV_LUMA, ME_YUV_I420: ME_YUV_I420}


class MVHeader(ctypes.Structure):
    _fields_ = [("magic", ctypes.c_char * 4), ("version", ctypes.c_uint16),
                ("flags", ctypes.c_uint16), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("block_size", ctypes.c_int32),
                ("search_range", ctypes.c_int32), ("cost", ctypes.c_int32),
                ("n_pairs", ctypes.c_uint32)]


def _path(p) -> bytes:
    return os.fsencode(p)


def _layout(layout) -> int:
    try:
        return _LAYOUT[layout]
    except KeyError:
        raise MEError(_lib.ME_EINVAL, f"unknown yuv layout {layout!r}") from None


def yuv_frame_count(path, width: int, height: int, layout="luma") -> int:
    n = int(_lib.lib().me_yuv_frame_count(_path(path), width, height, _layout(layout)))
    if n < 0:
        raise MEError(_lib.ME_EIO, f"cannot open {path}")
    return n


def read_luma(path, width: int, height: int, frame_index: int = 0, layout="luma",
              out: np.ndarray | None = None) -> np.ndarray:
    """Luma plane (height, width) uint8 of one frame (into `out` if given,
    e.g. a view of :func:`motionestimation_amd.pinned_frames`)."""
    if out is None:
        out = np.empty((height, width), np.uint8)
    if out.dtype != np.uint8 or out.shape != (height, width) or out.strides[1] != 1:
        raise MEError(_lib.ME_EINVAL, "out must be a (height, width) uint8 plane")
    check(_lib.lib().me_yuv_read_luma(_path(path), width, height, _layout(layout), frame_index,
                                      out.ctypes.data, out.strides[0]))
    return out


def write_yuv(path, data: np.ndarray, append: bool = False) -> None:
    data = np.ascontiguousarray(data, np.uint8)
    check(_lib.lib().me_yuv_write(_path(path), data.ctypes.data, data.nbytes, int(append)))


def write_mv(path, width: int, height: int, blk: int, span: int, cost, mv, block_cost=None,
             pairs=None) -> None:
    """mv: [npairs, nblocks, 2] (or [nblocks, 2] for one pair) int16;
    block_cost: matching uint32 or None; pairs: [(ref, cur), ...] or None
    (pair n = (n, n+1))."""
    mv = np.ascontiguousarray(mv, np.int16)
    if mv.ndim == 2:
        mv = mv[None]
    npairs = mv.shape[0]
    nb = num_blocks(width, height, blk)
    if mv.shape[1:] != (nb, 2):
        raise MEError(_lib.ME_EINVAL, f"mv shape {mv.shape} for {nb} blocks")
    cst = None
    if block_cost is not None:
        cst = np.ascontiguousarray(block_cost, np.uint32).reshape(npairs, nb)
    pr = None
    if pairs is not None:
        pr = np.ascontiguousarray(np.asarray(pairs, np.int32).reshape(npairs, 2))
    check(_lib.lib().me_mv_write(_path(path), width, height, blk, span, cost_code(cost),
                                 pr.ctypes.data if pr is not None else None, npairs,
                                 mv.ctypes.data, cst.ctypes.data if cst is not None else None))


def read_mv_header(path) -> dict:
    h = MVHeader()
    check(_lib.lib().me_mv_read_header(_path(path), ctypes.byref(h)))
    return {"width": h.width, "height": h.height, "block_size": h.block_size,
            "search_range": h.search_range, "cost": h.cost, "n_pairs": h.n_pairs,
            "has_cost": bool(h.flags & 1), "version": h.version}


def read_mv(path):
    """Returns (header dict, pairs int32 [npairs, 2], mv int16 [npairs, nblocks, 2],
    cost uint32 [npairs, nblocks] or None)."""
    hd = read_mv_header(path)
    nb = num_blocks(hd["width"], hd["height"], hd["block_size"])
    n = hd["n_pairs"]
    pairs = np.zeros((max(n, 1), 2), np.int32)
    mv = np.zeros((max(n, 1), max(nb, 1), 2), np.int16)
    cst = np.zeros((max(n, 1), max(nb, 1)), np.uint32) if hd["has_cost"] else None
    h = MVHeader()
    check(_lib.lib().me_mv_read(_path(path), ctypes.byref(h), pairs.ctypes.data, mv.ctypes.data,
                                cst.ctypes.data if cst is not None else None))
    return hd, pairs[:n], mv[:n, :nb], (cst[:n, :nb] if cst is not None else None)
