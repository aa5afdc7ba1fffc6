"""Deterministic synthetic Y-plane pairs (the reference's Beauty/Jockey frames are
absent: ``/root/reference/.MISSING_LARGE_BLOBS``).

Specification: splitmix64(seed) -> u8 uniform noise, 5x5 box
filter (edge replicate, rounded integer mean), ``cur`` = ``ref`` displaced by
(shift_x, shift_y) with edge replicate, plus uniform noise in [-2, 2], clipped
to [0, 255].  Pure numpy so it runs identically here and on the GPU box; the
frames are pinned by SHA-256 in ``tests/golden/manifest.json``.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# (width, height, seed, shift_x, shift_y) of the BASELINE.json synthetic configs.
CONFIGS = {
    "1080p": (1920, 1080, 1, 3, -3),
    "4k": (3840, 2160, 2, 17, -20),
    "8k": (7680, 4320, 3, 40, -27),
}


def splitmix64(seed: int, n: int, stream: int = 0) -> np.ndarray:
    """n outputs of splitmix64 started at ``seed`` (stream selects a disjoint
    counter range so ref noise and cur noise never share values)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64) + np.uint64(stream) * np.uint64(1 << 40)
        z = np.uint64(seed) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _box5(a: np.ndarray) -> np.ndarray:
    p = np.pad(a.astype(np.int64), 2, mode="edge")
    c = np.cumsum(np.cumsum(p, axis=0), axis=1)
    c = np.pad(c, ((1, 0), (1, 0)))
    h, w = a.shape
    s = c[5:5 + h, 5:5 + w] - c[0:h, 5:5 + w] - c[5:5 + h, 0:w] + c[0:h, 0:w]
    return ((s + 12) // 25).astype(np.uint8)


def shift_plane(a: np.ndarray, sx: int, sy: int) -> np.ndarray:
    """out[y, x] = a[clamp(y - sy), clamp(x - sx)]."""
    h, w = a.shape
    ys = np.clip(np.arange(h) - sy, 0, h - 1)
    xs = np.clip(np.arange(w) - sx, 0, w - 1)
    return a[ys[:, None], xs[None, :]]


def frame_pair(width: int, height: int, seed: int, shift_x: int, shift_y: int):
    """Return (ref, cur) as C-contiguous uint8 arrays of shape (height, width)."""
    n = width * height
    noise = (splitmix64(seed, n, 0) >> np.uint64(56)).astype(np.uint8).reshape(height, width)
    ref = _box5(noise)
    jitter = (splitmix64(seed, n, 1) % np.uint64(5)).astype(np.int16).reshape(height, width) - 2
    cur = np.clip(shift_plane(ref, shift_x, shift_y).astype(np.int16) + jitter, 0, 255)
    return np.ascontiguousarray(ref), np.ascontiguousarray(cur.astype(np.uint8))


def named_pair(name: str):
    w, h, seed, sx, sy = CONFIGS[name]
    return frame_pair(w, h, seed, sx, sy)


def sequence(width: int, height: int, n: int, seed: int, step_x: int, step_y: int,
             out: np.ndarray | None = None) -> np.ndarray:
    """n frames (n, height, width): frame k = the seed's box-filtered plane
    displaced by (k*step_x, k*step_y) plus its own [-2, 2] noise (stream k+1) --
    a camera pan for the frame-pair streaming path.  Written into `out` if given
    (e.g. pinned host memory)."""
    npx = width * height
    noise = (splitmix64(seed, npx, 0) >> np.uint64(56)).astype(np.uint8).reshape(height, width)
    base = _box5(noise)
    if out is None:
        out = np.empty((n, height, width), np.uint8)
    for k in range(n):
        jitter = (splitmix64(seed, npx, k + 1) % np.uint64(5)).astype(np.int16).reshape(
            height, width) - 2
        out[k] = np.clip(shift_plane(base, k * step_x, k * step_y).astype(np.int16) + jitter,
                         0, 255).astype(np.uint8)
    return out
