"""GPU: the context's one-search-at-a-time contract across streams, the
multi-device path inside the library (row stripes + one RCCL ncclGather,
csrc/me_api.hip multi_search), and bench.py's stripe mode end to end (the
north_star's 8-GPU split: one frame in row stripes, one gather per frame).

Tests that need two or more GPUs skip on a one-GPU box; the stripe-mode bench
is also run here as a 2-rank gloo rehearsal on one GPU (each rank searches its
stripe through libme_hip.so; the gather goes over gloo)."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O
import motionestimation_amd as me
from motionestimation_amd import synth

pytestmark = pytest.mark.gpu
NT = min(16, os.cpu_count() or 1)


def _ngpu():
    import torch
    return torch.cuda.device_count()


def _resident(ref, cur, blk):
    import torch
    h, w = ref.shape
    n = me.num_blocks(w, h, blk)
    return (torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda(),
            torch.full((n, 2), -7, dtype=torch.int16, device="cuda"),
            torch.zeros(n, dtype=torch.int32, device="cuda"))


@pytest.mark.parametrize("cost,blk,span,w,h", [
    ("ssd", 16, 32, 1920, 1080),   # MFMA path: shared prepass scratch
    ("ssd", 8, 24, 1280, 720),     # 8x8 MFMA path: merge keys + tile counters
    ("sad", 16, 16, 3840, 2160),   # qsad path with dynamic tile counters
])
def test_two_streams_one_context(cost, blk, span, w, h):
    """Two searches of one context enqueued back to back on two streams: the
    second waits for the first (they share the device's counters and scratch),
    so both fields are exact."""
    import torch
    a_ref, a_cur = synth.frame_pair(w, h, 31, 3, -2)
    b_ref, b_cur = synth.frame_pair(w, h, 32, -4, 5)
    with me.Engine(devices=[0]) as eng:
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for _ in range(2):  # and again, with the streams' order swapped
            ka, kb = _resident(a_ref, a_cur, blk), _resident(b_ref, b_cur, blk)
            torch.cuda.synchronize()
            for (rt, ct, mv, co), s in ((ka, s1), (kb, s2)):  # back to back, no host sync
                eng.full_search_device(rt, ct, blk, span, cost, mv, co,
                                       stream=ctypes.c_void_p(s.cuda_stream))
            torch.cuda.synchronize()
            for (ref, cur), (_, _, mv, co) in (((a_ref, a_cur), ka), ((b_ref, b_cur), kb)):
                omv, oco, _ = O.full_search(ref, cur, blk, span, cost, threads=NT)
                np.testing.assert_array_equal(mv.cpu().numpy(), omv)
                np.testing.assert_array_equal(co.cpu().numpy().view(np.uint32), oco)
            s1, s2 = s2, s1


@pytest.mark.skipif("_ngpu() < 2", reason="needs >= 2 GPUs (ncclCommInitAll + ncclGather)")
def test_multi_device_context_rccl_gather():
    """me_create over distinct devices 0..n-1: me_full_search stripes the frame
    across them and gathers with one ncclGather (me_api.hip multi_search)."""
    ref, cur = synth.frame_pair(1920, 1080, 7, 5, -3)
    n = _ngpu()
    for devs in sorted({2, n}):
        with me.Engine(devices=list(range(devs))) as eng:
            for cost, span in (("sad", 32), ("ssd", 32), ("sad", 7)):
                mv, c = eng.full_search(ref, cur, 16, span, cost)
                omv, oc, _ = O.full_search(ref, cur, 16, span, cost, threads=NT)
                np.testing.assert_array_equal(mv, omv, err_msg=f"{devs} devices {cost} S{span}")
                np.testing.assert_array_equal(c, oc)


def test_library_communicator_one_rank():
    """me_comm_init / me_gather_device (bench.py's RCCL exchange step) with a
    one-rank group: the gather lands the records bit for bit, on a side stream
    ordered by events; gathering before init and a second init fail loudly."""
    import torch
    with me.Engine(devices=[0]) as eng:
        src = torch.randint(-2**31, 2**31 - 1, (2, 1000), dtype=torch.int32, device="cuda")
        dst = torch.zeros((1, 2, 1000), dtype=torch.int32, device="cuda")
        with pytest.raises(me.MEError):
            eng.gather_device(src, dst)
        eng.comm_init(eng.comm_unique_id(), 1, 0)
        with pytest.raises(me.MEError):
            eng.comm_init(eng.comm_unique_id(), 1, 0)
        gs = torch.cuda.Stream()
        ev = torch.cuda.Event()
        ev.record()
        gs.wait_event(ev)
        eng.gather_device(src, dst, stream=ctypes.c_void_p(gs.cuda_stream))
        torch.cuda.synchronize()
        assert torch.equal(dst[0], src)


def test_comm_check_one_rank():
    """me_comm_check (failure detection of the exchange): clean after a
    gather on a one-rank group; when the stream's work outlasts the timeout it
    returns ME_ECOMM and aborts the communicator, the stream still drains,
    every later gather or check fails loudly instead of hanging, and a new
    me_comm_init recovers the context."""
    import torch
    with me.Engine(devices=[0]) as eng:
        with pytest.raises(me.MEError):  # no communicator yet
            eng.comm_check(1000)
        eng.comm_init(eng.comm_unique_id(), 1, 0)
        src = torch.arange(4096, dtype=torch.int32, device="cuda")
        dst = torch.zeros((1, 4096), dtype=torch.int32, device="cuda")
        eng.gather_device(src, dst)
        eng.comm_check(10_000)
        assert torch.equal(dst[0], src)
        # ~10 ms of searches ahead of the check, and a zero timeout: a "stalled" exchange
        w, h = 1920, 1080
        ref = torch.randint(0, 256, (16, h, w), dtype=torch.uint8, device="cuda")
        cur = torch.randint(0, 256, (16, h, w), dtype=torch.uint8, device="cuda")
        nb = me.num_blocks(w, h, 16)
        mv = torch.empty((16 * nb, 2), dtype=torch.int16, device="cuda")
        co = torch.empty(16 * nb, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        for _ in range(10):
            eng.search_batch_device(ref, 0, cur, 0, w, h, 16, 32, "sad", 0, (h + 15) // 16, mv, co)
        eng.gather_device(src, dst)
        with pytest.raises(me.MEError) as e:
            eng.comm_check(0)
        assert e.value.status == me.ME_ECOMM and "aborted" in str(e.value)
        torch.cuda.synchronize()  # the aborted rank's stream drains
        with pytest.raises(me.MEError) as e:
            eng.gather_device(src, dst)
        assert e.value.status == me.ME_ECOMM
        with pytest.raises(me.MEError) as e:
            eng.comm_check(1000)
        assert e.value.status == me.ME_ECOMM
        eng.device_check()
        # a new communicator (fresh id, every rank) makes the context usable again
        eng.comm_init(eng.comm_unique_id(), 1, 0)
        dst.zero_()
        src1 = src + 1
        eng.gather_device(src1, dst)
        eng.comm_check(10_000)
        assert torch.equal(dst[0], src1)


def _bench_ranks(nproc, backend, extra=()):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", "--master-port=29731",
           os.path.join(O.REPO, "bench.py"), "--gpus", str(nproc), "--dist-backend", backend,
           "--steps", "4", "--warmup", "1", "--no-cpu", "--no-ssd", "--no-stream", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _bench_no_launcher(nproc, backend, extra=()):
    """bench.py --gpus N with no torch.distributed.run around it (the driver's
    own command line): bench.py starts the N ranks itself."""
    cmd = [sys.executable, os.path.join(O.REPO, "bench.py"), "--gpus", str(nproc),
           "--dist-backend", backend, "--steps", "4", "--warmup", "1", "--no-cpu", "--no-ssd",
           "--no-stream", *extra]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=115, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    return json.loads(lines[0])


def _check_stripe_line(d, nproc):
    assert d["n_gpus"] == nproc and d["scaling"] == "strong"
    assert d["config"]["parallelism"] == f"stripe{nproc}"
    assert d["stripe_gather_parity"] is True
    assert d["stripe_4k"]["stripe_gather_parity"] is True
    # the line verifies its own timed work: gathered fields == batched search
    # == the committed per-frame pins, every rank's device check clean
    assert d["parity"] is True, d["parity_legs"]
    for leg in (d["parity_legs"]["timed_step"], d["stripe_4k"]["parity"]):
        assert leg["ok"] and leg["pinned_frames"] == leg["pinned_equal"] == leg["frames"], leg
    assert d["stripe_4k"]["parallelism"] == f"stripe{nproc}"
    assert d["value"] > 0 and d["stripe_4k"]["value"] > 0


def test_bench_stripe_mode_two_ranks_gloo_rehearsal():
    """bench.py --gpus 2 in its N > 1 default (stripe mode) with two ranks on
    one GPU over gloo: each rank's stripe goes through libme_hip.so and the
    gathered 1080p and 4K fields equal a full-frame search."""
    _check_stripe_line(_bench_ranks(2, "gloo"), 2)


def test_bench_spawns_its_own_ranks_gloo():
    """`python bench.py --gpus 2` with no launcher (how the driver runs it):
    two ranks, started by bench.py itself, in stripe mode with gather parity
    for the 1080p line and the nested 4K record (gloo: both ranks on one GPU)."""
    _check_stripe_line(_bench_no_launcher(2, "gloo"), 2)


@pytest.mark.parametrize("nproc", [4, 8])
def test_bench_spawns_n_ranks_gloo(nproc):
    """The SCALE shapes rehearsed on one GPU: `python bench.py --gpus N` (N = 4,
    8) with no launcher starts N ranks; each searches stripe (r + f) mod N of
    frame f of the 16-frame step, rank 0 reassembles every frame, and the 1080p
    and 4K fields equal the batched search and the pins (gloo carries the
    gather: RCCL needs one GPU per rank)."""
    _check_stripe_line(_bench_no_launcher(nproc, "gloo", ("--ramp-ms", "10")), nproc)


def test_bench_stripe_mode_rccl_one_rank():
    """bench.py's RCCL stripe path end to end on one GPU: torch.distributed.run
    with one rank, the unique id broadcast, me_comm_init, and every frame's
    me_gather_device (1080p and the nested 4K record), gathered fields equal to
    a full-frame search."""
    d = _bench_ranks(1, "nccl", ("--mode", "stripe"))
    _check_stripe_line(d, 1)
    assert "me_gather_device" in d["config"]["gather"]
    assert "me_gather_device" in d["stripe_4k"]["gather"]


def _live_streams(log):
    """Streams a process had created and not destroyed while its search
    kernels were launched (the most at any such launch), from the HIP
    runtime's own API log (AMD_LOG_LEVEL=3): creations return 'stream:0x...',
    destructions name it, launches log 'ShaderName : <kernel>'.  (RCCL's proxy
    thread creates and destroys one more stream during communicator setup,
    before any search.)"""
    import re
    live, peak = set(), 0
    for line in log.splitlines():
        m = re.search(r"hipStreamCreate\w*: Returned hipSuccess : stream:(0x[0-9a-f]+)", line)
        if m:
            live.add(m.group(1))
            continue
        m = re.search(r"hipStreamDestroy \( stream:(0x[0-9a-f]+)", line)
        if m:
            live.discard(m.group(1))
            continue
        if "ShaderName : " in line and "me::" in line:
            peak = max(peak, len(live))
    return peak


def test_rccl_rank_stream_budget():
    """A bench.py RCCL stripe rank holds at most 4 created HIP streams
    (GPU_MAX_HW_QUEUES = 4 hardware queues per process): torch's stream (the
    searches and the gather) and the one RCCL communicator's (the library's
    ncclGather).  The library creates none for device entry points (its own
    stream is lazy), and torch's process group is gloo (the control plane), so
    there is no second communicator (round 4: torch's "nccl" group + the
    library's communicator + the context stream).  Counted from the HIP
    runtime's API log of the one-rank run."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=29733", os.path.join(O.REPO, "bench.py"),
           "--gpus", "1", "--mode", "stripe", "--steps", "3", "--warmup", "1", "--no-cpu",
           "--no-4k", "--ramp-ms", "5"]
    env = dict(os.environ, OMP_NUM_THREADS="1", AMD_LOG_LEVEL="3")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=115, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert "me_gather_device" in d["config"]["gather"]
    peak = _live_streams(r.stderr)
    assert 1 <= peak <= 4, f"{peak} live streams"


@pytest.mark.skipif("_ngpu() < 2", reason="needs >= 2 GPUs (one RCCL rank per GPU)")
def test_bench_stripe_mode_rccl():
    """The same over RCCL, one rank per GPU (asynchronous gathers overlapping
    the next frame's search)."""
    n = min(_ngpu(), 8)
    for k in sorted({2, n}):
        d = _bench_ranks(k, "nccl")
        _check_stripe_line(d, k)
        assert "me_gather_device" in d["config"]["gather"]
