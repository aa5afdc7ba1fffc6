"""Per-context kernel path (me_ctx_set_kernel_path / me_ctx_last_search_path).

include/me.h allows one host thread per context; two contexts on two threads
must be able to run different kernel families at once, and each must report
its own.  The searches are the reference's 16x16 MSE search
(souravBhat/MotionEstimation src/cpu/main.c:18-82) as integer SSD, checked
against the oracle bit for bit.
"""
import os
import threading

import numpy as np
import pytest

import oracle_lib as O
import motionestimation_amd as me
from motionestimation_amd import synth

pytestmark = pytest.mark.gpu
NT = min(16, os.cpu_count() or 1)


def _pair(seed, h=272, w=352):
    rng = np.random.default_rng(seed)
    ref = synth._box5(rng.integers(0, 256, (h, w), dtype=np.uint8))
    cur = np.clip(synth.shift_plane(ref, 3, -2).astype(int) + rng.integers(-3, 4, (h, w)), 0,
                  255).astype(np.uint8)
    return ref, cur


def test_two_contexts_two_threads_own_paths():
    """Context A runs the VALU kernels, context B the band-walk MFMA kernel,
    context C the prepass pair, concurrently from three threads while the
    process-wide path stays 'auto'; every search's reported family is the
    context's own and every field equals the oracle's."""
    pairs = {k: _pair(s) for k, s in (("valu", 1), ("lean", 2), ("prepass", 3))}
    want = {"valu": "valu", "lean": "mfma_bandwalk", "prepass": "mfma_prepass"}
    oracle = {k: O.full_search(r, c, 16, 32, "ssd", threads=NT)[:2] for k, (r, c) in pairs.items()}
    me.set_kernel_path("auto")
    engines = {k: me.Engine(devices=[0]) for k in pairs}
    errors = []
    start = threading.Barrier(len(pairs))

    def run(k):
        try:
            eng = engines[k]
            eng.set_kernel_path(k)
            ref, cur = pairs[k]
            start.wait()
            for _ in range(12):
                mv, c = eng.full_search(ref, cur, 16, 32, "ssd")
                got = eng.last_search_path()
                if got != want[k]:
                    errors.append(f"{k}: reported {got}, want {want[k]}")
                    return
                np.testing.assert_array_equal(mv, oracle[k][0])
                np.testing.assert_array_equal(c, oracle[k][1])
        except Exception as e:  # noqa: BLE001 -- reported on the main thread
            errors.append(f"{k}: {e!r}")

    th = [threading.Thread(target=run, args=(k,)) for k in pairs]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    try:
        assert not any(t.is_alive() for t in th), "a search thread did not finish"
        assert not errors, errors
        # back to the process-wide path: a SAD search is VALU on every path,
        # an SSD search follows the global value again
        eng = engines["valu"]
        eng.set_kernel_path(None)
        me.set_kernel_path("prepass")
        ref, cur = pairs["valu"]
        mv, c = eng.full_search(ref, cur, 16, 32, "ssd")
        assert eng.last_search_path() == "mfma_prepass"
        np.testing.assert_array_equal(mv, oracle["valu"][0])
        # the other contexts still report their own last search
        assert engines["lean"].last_search_path() == "mfma_bandwalk"
        assert engines["prepass"].last_search_path() == "mfma_prepass"
    finally:
        me.set_kernel_path("auto")
        for e in engines.values():
            e.close()


def test_ctx_path_argument_checks():
    with me.Engine(devices=[0]) as eng:
        assert eng.last_search_path() == "none"
        with pytest.raises(me.MEError):
            eng.set_kernel_path("bogus")
        from motionestimation_amd import _lib
        assert _lib.lib().me_ctx_set_kernel_path(eng._h, 99) == _lib.ME_EINVAL
        assert _lib.lib().me_ctx_last_search_path(eng._h, 5) == -1
        assert _lib.lib().me_ctx_last_search_path(None, 0) == -1


def test_multi_device_context_path_on_worker_threads():
    """A context over the device list [0, 0] runs me_search_pairs on one host
    worker per context device; the workers plan with the context's own path
    and record it per device (round 6: their per-device error contexts first
    indexed the wrong context's slots and crashed)."""
    frames = [_pair(s, 208, 256)[0] for s in range(5)]
    pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 0), (1, 3)]
    me.set_kernel_path("auto")
    with me.Engine(devices=[0, 0]) as eng:
        eng.set_kernel_path("prepass")
        mv, c = eng.search_pairs(frames, pairs, 16, 16, "ssd")
        assert eng.last_search_path(0) == "mfma_prepass", eng.last_search_path(0)
        assert eng.last_search_path(1) == "mfma_prepass", eng.last_search_path(1)
        for i, (a, b) in enumerate(pairs):
            omv, oc, _ = O.full_search(frames[a], frames[b], 16, 16, "ssd", threads=NT)
            np.testing.assert_array_equal(mv[i], omv, err_msg=f"pair {i}")
            np.testing.assert_array_equal(c[i], oc, err_msg=f"pair {i}")
