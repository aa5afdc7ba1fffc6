"""GPU: whole-frame bit-exact pins at the largest BASELINE configs.

tests/golden/make_big_golden.py hashed the full per-block record stream of
  * BASELINE configs[4] (8K 7680x4320, 8x8, +-128) under the REAL reference
    (oracle/_ref/ref_dump: findBestBlkMse, src/cpu/main.c:67-82, every one of the
    518,400 blocks): int32 mvx, int32 mvy, float32 mse;
  * the same frame and BASELINE configs[3] (4K, 16x16, +-64) under the SAD
    restatement (oracle/me_oracle.c): int16 mvx, int16 mvy, uint32 sad.
Here the GPU searches the same synthetic frames (pinned by SHA-256 in the
manifest) and must reproduce each hash exactly; a mismatch names the block-row
bands that differ.  The SSD field is checked on the default (matrix-core) path
and on the VALU kernels.
"""
import hashlib

import numpy as np
import pytest

import motionestimation_amd as me
from motionestimation_amd import synth

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _case(manifest, name):
    return [c for c in manifest["big_cases"] if c["name"] == name][0]


def _check(rec, case):
    if hashlib.sha256(rec.tobytes()).hexdigest() == case["sha256"]:
        return
    w, h, blk, bands = case["width"], case["height"], case["blk"], case["bands"]
    nbx, nby = (w + blk - 1) // blk, (h + blk - 1) // blk
    bad = []
    for b, want in enumerate(case["band_sha256"]):
        r0, r1 = nby * b // bands, nby * (b + 1) // bands
        if hashlib.sha256(rec[r0 * nbx:r1 * nbx].tobytes()).hexdigest() != want:
            bad.append(f"band {b} (block rows {r0}..{r1 - 1})")
    pytest.fail(f"{case['name']}: record stream differs from the pinned hash in {bad or 'no band (?)'}")


def _ssd_records(mv, cost, blk, w, h):
    """The reference's record: int32 mvx, int32 mvy, float32 (float)SSD / (w*h)."""
    nbx, nby = (w + blk - 1) // blk, (h + blk - 1) // blk
    bw = np.minimum(blk, w - np.arange(nbx) * blk)
    bh = np.minimum(blk, h - np.arange(nby) * blk)
    area = (bh[:, None] * bw[None, :]).reshape(-1).astype(np.float32)
    rec = np.empty((len(mv), 3), np.int32)
    rec[:, :2] = mv
    rec[:, 2] = (cost.astype(np.float32) / area).view(np.int32)
    return rec


def _sad_records(mv, cost):
    rec = np.empty((len(mv), 8), np.uint8)
    rec[:, :4] = np.ascontiguousarray(mv, np.int16).view(np.uint8).reshape(-1, 4)
    rec[:, 4:] = np.ascontiguousarray(cost, np.uint32).view(np.uint8).reshape(-1, 4)
    return rec


@pytest.fixture(scope="module")
def frames_8k():
    return synth.named_pair("8k")


@pytest.mark.parametrize("path", ["auto", "valu"])
def test_8k_b8_s128_ssd_matches_reference_every_block(engine, manifest, frames_8k, path):
    case = _case(manifest, "big_8k_b8_s128_ssd")
    ref, cur = frames_8k
    me.set_kernel_path(path)
    try:
        mv, cost = engine.full_search(ref, cur, 8, 128, "ssd")
    finally:
        me.set_kernel_path("auto")
    _check(_ssd_records(mv, cost, 8, 7680, 4320), case)


def test_8k_b8_s128_sad_every_block(engine, manifest, frames_8k):
    ref, cur = frames_8k
    mv, cost = engine.full_search(ref, cur, 8, 128, "sad")
    _check(_sad_records(mv, cost), _case(manifest, "big_8k_b8_s128_sad"))


def test_4k_b16_s64_sad_every_block(engine, manifest):
    ref, cur = synth.named_pair("4k")
    mv, cost = engine.full_search(ref, cur, 16, 64, "sad")
    _check(_sad_records(mv, cost), _case(manifest, "big_4k_b16_s64_sad"))
