"""libme_hip.so loads and exports every symbol include/me.h declares; host-only
helpers (no GPU) behave like the reference's tiling and counting."""
import ctypes
import os
import re

import numpy as np
import pytest

import motionestimation_amd as me
from motionestimation_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(REPO, "include", "me.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(me_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_header_symbols():
    L = _lib.lib()
    syms = _declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
        assert s in _lib._SIGS, f"{s} has no ctypes signature"


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_status_strings():
    assert "gfx950" in me.version()
    L = _lib.lib()
    assert L.me_status_str(0) == b"ok"
    assert L.me_status_str(1) == b"invalid argument"


def test_num_blocks_matches_reference_tiling():
    for (w, h, b) in [(352, 288, 16), (1920, 1080, 16), (100, 75, 16), (7, 5, 16), (352, 288, 7)]:
        assert me.num_blocks(w, h, b) == ((w + b - 1) // b) * ((h + b - 1) // b)
    assert me.num_blocks(0, 10, 4) == 0


def test_candidate_count_matches_oracle():
    import oracle_lib as O
    for args in [(352, 288, 8, 12), (1920, 1080, 16, 32), (100, 75, 16, 9), (7, 5, 16, 4),
                 (3840, 2160, 16, 64), (352, 288, 7, 15)]:
        assert me.candidate_count(*args) == O.candidate_count(*args), args


def test_stripe_plan_is_balanced_partition():
    for (w, h, b, s, n) in [(1920, 1080, 16, 32, 8), (3840, 2160, 16, 64, 8), (352, 288, 16, 16, 3),
                            (1920, 1080, 16, 32, 1), (64, 48, 16, 7, 8)]:
        bounds = me.plan_stripes(w, h, b, s, n)
        nby = (h + b - 1) // b
        assert bounds[0] == 0 and bounds[-1] == nby
        assert all(bounds[i] <= bounds[i + 1] for i in range(n))
        if nby >= n:
            assert all(bounds[i] < bounds[i + 1] for i in range(n)), bounds
        if n == 8 and h >= 1080:
            # each shard within one block row of the ideal candidate share
            rows = [me.candidate_count(w, min(h, (r + 1) * b), b, s) for r in range(nby)]
            assert max(bounds[i + 1] - bounds[i] for i in range(n)) <= nby // n + 2


def test_create_without_gpu_fails_cleanly():
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(me.MEError):
        me.Engine()


def test_prediction_frame_matches_oracle_tiling():
    import oracle_lib as O  # noqa: F401
    f = np.zeros((75, 100), np.uint8)
    pf = me.create_prediction_frame(f, 100, 75, 16)
    assert pf.num_blks == 7 * 5
    last = pf.blks[-1]
    assert (last.width, last.height, last.bottom_right_x, last.bottom_right_y) == (4, 11, 99, 74)
    assert pf.blks[0].motion_vectorY == -1000
