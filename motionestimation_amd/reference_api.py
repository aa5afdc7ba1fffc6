"""The reference's own interface for the hot path, same names and meaning,
served by the GPU engine.

Reference (souravBhat/MotionEstimation):
  block struct                 src/common/block.h:6-19, createBlk block.c:3-13
  predictionFrame              src/common/prediction_frame.h:8-16
  createPredictionFrame        src/common/prediction_frame.c:3-25
  findBestBlkMse (per block)   src/cpu/main.c:67-82  -> find_best_blk_mse
  findBestBlkSSIM (per block)  src/cpu/main_ssim.c:15-29 -> find_best_blk_ssim
  thread-pool dispatch         src/cpu/main.c:144-158 -> find_best_blks (whole frame)
  motionCompensatedFrame       src/common/utils.c:102-134
  frameDiff / imagePSNR        src/common/utils.c:94-100 / :137-164
Error behaviour: the reference prints and exit()s; here an MEError (or
ValueError for a missing best match, utils.c:105-108) is raised instead.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .engine import Engine


@dataclass
class Block:
    idx_x: int
    idx_y: int
    top_left_x: int
    top_left_y: int
    bottom_right_x: int
    bottom_right_y: int
    width: int
    height: int
    is_best_match_found: int = 0
    motion_vectorX: int = 0
    motion_vectorY: int = -1000  # block.c:12


@dataclass
class PredictionFrame:
    frame: np.ndarray
    width: int
    height: int
    blk_dim: int
    num_blks: int
    blks: list = field(default_factory=list)


def create_prediction_frame(frame, width: int, height: int, blk_dim: int) -> PredictionFrame:
    """createPredictionFrame: ceil tiling, partial blocks on the edges."""
    frame = np.asarray(frame).reshape(height, width)
    nbx = (width + blk_dim - 1) // blk_dim
    nby = (height + blk_dim - 1) // blk_dim
    blks = []
    for i in range(nbx * nby):
        bx, by = i % nbx, i // nbx
        tlx, tly = bx * blk_dim, by * blk_dim
        w = blk_dim if tlx + blk_dim < width else width - tlx
        h = blk_dim if tly + blk_dim < height else height - tly
        blks.append(Block(bx, by, tlx, tly, tlx + w - 1, tly + h - 1, w, h))
    return PredictionFrame(frame, width, height, blk_dim, nbx * nby, blks)


_default_engine = None


def _engine(engine):
    global _default_engine
    if engine is not None:
        return engine
    if _default_engine is None:
        _default_engine = Engine()
    return _default_engine


def find_best_blks(pf: PredictionFrame, reference_frame, extra_span: int, cost="ssd",
                   engine=None) -> np.ndarray:
    """All blocks of pf at once (the thread-pool loop of main.c:144-158).
    Fills motion_vectorX/Y and is_best_match_found = 1 on every block and
    returns the per-block MSE (SSD / (w*h) as float32, the reference's score),
    SAD, or for cost="ssim" the reference's SSIM score (float32; 0 with MV
    (0, 0) where no candidate scores above 0, ssim.c:87-104)."""
    ref = np.asarray(reference_frame).reshape(pf.height, pf.width).astype(np.uint8)
    cur = np.asarray(pf.frame).reshape(pf.height, pf.width).astype(np.uint8)
    mv, cst = _engine(engine).full_search(ref, cur, pf.blk_dim, extra_span, cost)
    for b, (mx, my) in zip(pf.blks, mv.tolist()):
        b.motion_vectorX, b.motion_vectorY, b.is_best_match_found = mx, my, 1
    if cost in ("ssd", "mse", 0):
        area = np.array([b.width * b.height for b in pf.blks], np.float32)
        return cst.astype(np.float32) / area
    if cost in ("ssim", 2):
        return cst.view(np.float32)
    return cst


def find_best_blk_mse(pf: PredictionFrame, reference_frame, blk: Block, extra_span: int,
                      engine=None) -> float:
    """findBestBlkMse for one block (kept for interface parity; it searches the
    frame on the GPU and picks this block's result)."""
    scores = find_best_blks(pf, reference_frame, extra_span, "ssd", engine)
    i = blk.idx_y * ((pf.width + pf.blk_dim - 1) // pf.blk_dim) + blk.idx_x
    src = pf.blks[i]
    blk.motion_vectorX, blk.motion_vectorY = src.motion_vectorX, src.motion_vectorY
    blk.is_best_match_found = 1
    return float(scores[i])


def find_best_blk_ssim(pf: PredictionFrame, reference_frame, blk: Block, extra_span: int,
                       engine=None) -> float:
    """findBestBlkSSIM for one block (main_ssim.c:15-29): the best SSIM score,
    MV written into blk (the search runs over the frame on the GPU)."""
    scores = find_best_blks(pf, reference_frame, extra_span, "ssim", engine)
    i = blk.idx_y * ((pf.width + pf.blk_dim - 1) // pf.blk_dim) + blk.idx_x
    src = pf.blks[i]
    blk.motion_vectorX, blk.motion_vectorY = src.motion_vectorX, src.motion_vectorY
    blk.is_best_match_found = 1
    return float(scores[i])


def mv_field(pf: PredictionFrame) -> np.ndarray:
    for i, b in enumerate(pf.blks):
        if b.is_best_match_found != 1:  # utils.c:105-108 exits here
            raise ValueError("Trying to create compensation frame without best match, "
                             f"value = {b.is_best_match_found} for block {i}")
    return np.array([[b.motion_vectorX, b.motion_vectorY] for b in pf.blks], np.int16)


def motion_compensated_frame(pf: PredictionFrame, ref_frame, engine=None) -> np.ndarray:
    ref = np.asarray(ref_frame).reshape(pf.height, pf.width).astype(np.uint8)
    return _engine(engine).motion_compensate(ref, pf.blk_dim, mv_field(pf))


def frame_diff(a, b) -> np.ndarray:
    return np.abs(np.asarray(a, np.int32) - np.asarray(b, np.int32)).astype(np.uint8)


def output_planes(pf: PredictionFrame, ref_frame, engine=None):
    """[ref, cur, mc, |ref-cur|, |mc-cur|] (main.c:161-168) and imagePSNR(mc, cur)."""
    ref = np.asarray(ref_frame).reshape(pf.height, pf.width).astype(np.uint8)
    cur = np.asarray(pf.frame).reshape(pf.height, pf.width).astype(np.uint8)
    return _engine(engine).compensate_planes(ref, cur, pf.blk_dim, mv_field(pf))
