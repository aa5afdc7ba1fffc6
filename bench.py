#!/usr/bin/env python3
"""bench.py -- full-search block matching throughput on MI355X.

Metric (BASELINE.json): 16x16 SAD candidates/sec at 1080p +-32; achieved HBM
GB/s vs roofline.  One step = full searches of a batch of 1920x1080 Y-frame
pairs (B=16, S=32, SAD, 33,188,832 exact candidates per frame), inputs
resident in HBM before the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode auto|frames|stripe]
                  [--config 1080p|4k|8k] [--cost sad|ssd] [--no-cpu]

A step is a batch of --frames-per-step F frames (default 16), searched in one
launch per rank (me_full_search_batch_device; in stripe mode the rank's F
stripes, me_search_stripes_device).
--mode stripe (the default for N > 1, north_star's split): the step's F frames
  are each split into cost-balanced block-row stripes, one per rank, each rank
  holding only its stripes + S-row ref halos; the per-stripe MV records of all
  F frames are gathered to rank 0 with one RCCL gather per step inside the
  timed region (strong scaling).  Double-buffered records.
--mode frames (the default for N = 1, where it is the same search): each rank
  searches its own F frame pairs per step: weak scaling, no collective.
Every line also carries `stripe_4k`: BASELINE configs[3] (4K +-64) in stripe
mode on the same ranks, with its gather parity.
For N > 1: one process per GPU over RCCL.  Under torch.distributed.run
(WORLD_SIZE set) the ranks are the launcher's; without a launcher bench.py
starts `torch.distributed.run --nproc-per-node N` itself as a child before
anything touches the GPU and forwards its line (launch_ranks; fewer visible
GPUs than RCCL ranks is an error, never an n_gpus = 1 line).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "16×16 SAD candidates/sec at 1080p ±32; achieved HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
MAX_JOBS = 32                # jobs per kernel launch (csrc/me_kernels.h): SAD batches share launches
VALU_PEAK_ABSDIFF = 157.3e12  # 256 CU x 64 lanes x 2.4 GHz x 4 |a-b| per op (measured: profiles/)
VALU_PEAK_LANE = 78.6e12      # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (wave64 issues over 2 clocks)
I8_PEAK_TOPS = 5000.0         # MI355X_MICROARCH.md: dense I8 MFMA = 2x BF16 (2.5 PF) per clock
CONFIGS = {  # name -> (synth config, block, range)
    "1080p": ("1080p", 16, 32),
    "4k": ("4k", 16, 64),
    "8k": ("8k", 8, 128),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["auto", "frames", "stripe"], default="auto",
                    help="auto: frames at N = 1, stripe at N > 1")
    ap.add_argument("--config", choices=list(CONFIGS), default="1080p")
    ap.add_argument("--cost", choices=["sad", "ssd", "ssim"], default="sad")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-ssd", action="store_true",
                    help="skip the SSD (matrix-core) line beside a SAD run")
    ap.add_argument("--no-ssim", action="store_true",
                    help="skip the SSIM-cost leg beside a 1080p SAD run")
    ap.add_argument("--no-stream", action="store_true",
                    help="skip the host frame-pair streaming leg (PCIe-inclusive, not `value`)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the main CPU-baseline leg (default: the process's cgroup "
                         "CPU quota, cpu.max, rounded down; 16 if none is set)")
    ap.add_argument("--no-4k", action="store_true", help="skip the nested stripe_4k record")
    ap.add_argument("--no-single", action="store_true",
                    help="skip the single_frame record (one frame per launch, for comparison)")
    ap.add_argument("--graph", action="store_true",
                    help="stripe mode over RCCL: replay search + gather as one captured hipGraph "
                         "per step instead of two enqueues (measured slower on one GPU)")
    ap.add_argument("--ramp-ms", type=float, default=100.0,
                    help="untimed steps for this long before the W warmup steps (GPU clock ramp)")
    ap.add_argument("--frames-per-step", type=int, default=16,
                    help="frames searched per step: one batched launch per rank "
                         "(me_full_search_batch_device) and, in stripe mode, one gather per step")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="the data exchange: nccl = the library's RCCL gather (production); gloo "
                         "= torch.distributed.gather, only to rehearse N ranks on one GPU.  "
                         "torch's own process group (control plane) is gloo either way")
    ap.add_argument("--torch-pg", choices=["gloo", "nccl"], default="gloo",
                    help="torch.distributed's own process group (control plane); nccl only to "
                         "A/B the round-4 configuration (a second RCCL communicator per rank)")
    ap.add_argument("--comm-timeout-ms", type=int, default=60000,
                    help="RCCL ranks: bounded wait for a step's searches + gather (me_comm_check); "
                         "past it the rank aborts its communicator and exits non-zero")
    return ap.parse_args()


def _block_candidates(w, h, blk, span, bx, by):
    """Exact candidates of one block under the reference's clamping (main.c:73-76)."""
    tlx, tly = bx * blk, by * blk
    bw, bh = min(blk, w - tlx), min(blk, h - tly)
    nx = min(span, w - bw - tlx) - max(-span, -tlx) + 1
    ny = min(span, h - bh - tly) - max(-span, -tly) + 1
    return nx * ny


def exact_absdiffs(w, h, blk, span, row0=0, row1=None):
    """Exact |a-b| (or multiply-add) count of block rows [row0, row1): every
    block's candidates (main.c:53-54, 73-76) times its own w*h pixels (edge
    blocks are partial, prediction_frame.c:21-22).  1080p 16x16 +-32:
    8,463,799,296."""
    nbx, nby = (w + blk - 1) // blk, (h + blk - 1) // blk
    row1 = nby if row1 is None else row1
    bx = np.arange(nbx, dtype=np.int64)
    by = np.arange(row0, row1, dtype=np.int64)
    tlx, tly = bx * blk, by * blk
    bw, bh = np.minimum(blk, w - tlx), np.minimum(blk, h - tly)
    nx = np.minimum(span, w - bw - tlx) - np.maximum(-span, -tlx) + 1
    ny = np.minimum(span, h - bh - tly) - np.maximum(-span, -tly) + 1
    return int((nx * bw).sum() * (ny * bh).sum())


def cgroup_cpu_quota():
    """The process's CPU quota from its cgroup: (source text, CPUs as a float,
    or None when unlimited / unreadable).  cgroup v2: the smallest cpu.max
    ("<quota> <period>" or "max <period>") from the process's cgroup up to the
    mounted root; else v1 cpu.cfs_quota_us / cpu.cfs_period_us."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = next((l.strip().split(":", 2)[2] for l in f if l.startswith("0::")), "/")
    except (OSError, IndexError):
        rel = "/"
    best, seen = None, []
    d = os.path.join("/sys/fs/cgroup", rel.lstrip("/")).rstrip("/")
    while d.startswith("/sys/fs/cgroup"):
        try:
            with open(os.path.join(d, "cpu.max")) as f:
                raw = f.read().strip()
            seen.append(f"{d}/cpu.max: {raw}")
            q, _, p = raw.partition(" ")
            if q != "max" and p:
                cpus = int(q) / int(p)
                best = cpus if best is None else min(best, cpus)
        except (OSError, ValueError):
            pass
        d = os.path.dirname(d)
    if seen:
        return "; ".join(seen), best
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return f"cgroup v1 cfs_quota_us {q} period {p}", (q / p if q > 0 else None)
    except (OSError, ValueError):
        return None, None


def cpu_baselines(ref, cur, blk, span, cost, threads, cands):
    """Rank 0, N=1 only: the oracle restatement (port) timed on the host cores
    on the same frame pair, and the reference's own binary (oracle/_ref/mes,
    MSE cost, its hard-coded 100-thread pool) when it was built.  Returns
    (record, the port's field (mv, cost) of the whole frame or None): the field
    is the checker of the timed step's frame 0 (bench.verify_fields)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    h, w = ref.shape
    nbx, nby = (w + blk - 1) // blk, (h + blk - 1) // blk
    begin, end, what = 0, nbx * nby, "the full"
    if cost == "ssim":  # ~40x the work per candidate: a bounded sample of 4 middle block rows
        r0 = max(0, nby // 2 - 2)
        begin, end = r0 * nbx, min(nby, r0 + 4) * nbx
        what = f"block rows {r0}..{min(nby, r0 + 4) - 1} of the"
        cands = sum(_block_candidates(w, h, blk, span, i % nbx, i // nbx)
                    for i in range(begin, end))
    quota_raw, quota = cgroup_cpu_quota()
    if threads is None:
        threads = max(1, int(quota)) if quota else 16
    field = []

    def port(nthreads, variant="", reps=5):
        """median seconds of `reps` oracle searches over blocks [begin, end)"""
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = O.full_search(ref, cur, blk, span, cost, threads=nthreads, begin=begin, end=end,
                              variant=variant)
            times.append(time.perf_counter() - t0)
            if not field:
                field.append(r[:2])
        return statistics.median(times)

    med = port(threads)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    affinity = len(os.sched_getaffinity(0))
    out = {"value": cands / med, "unit": "candidates/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model, "host_cpus": os.cpu_count(), "affinity_cpus": affinity,
           "cgroup_cpu_quota": {"cpus": quota, "source": quota_raw},
           "sample": f"{what} {w}x{h} B{blk} +-{span} {cost.upper()} frame, "
                     f"oracle/me_oracle.c -O2, {threads} pthreads, median of 5 ({med*1e3:.1f} ms)"}
    # SURVEY §8d's other legs: the port with the reference's 100-thread pool
    # (main.c:144) and with one thread per CPU of this process's affinity mask,
    # and the port built without optimisation (as src/cpu/run.sh:4 builds).
    legs = []
    for n in sorted({100, affinity}):
        m = port(n, reps=3)
        legs.append({"threads": n, "value": cands / m, "unit": "candidates/s",
                     "sample": f"same blocks, -O2, {n} pthreads, median of 3 ({m*1e3:.1f} ms)"})
    out["port_threads"] = legs
    m = port(threads, variant="O0", reps=3)
    out["port_O0"] = {"threads": threads, "value": cands / m, "unit": "candidates/s",
                      "sample": f"same blocks, oracle/liboracle_O0.so (-O0), {threads} pthreads, "
                                f"median of 3 ({m*1e3:.1f} ms)"}
    # the reference binary at -O2, and as src/cpu/run.sh:4 builds it (-O0)
    for key, name, opt in (("reference_binary", "mes", "-O2"), ("reference_binary_O0", "mes_O0", "-O0")):
        mes = os.path.join(REPO, "oracle", "_ref", name)
        if not os.path.exists(mes) or cost == "ssim":
            continue
        with tempfile.TemporaryDirectory() as td:
            rp, cp = os.path.join(td, "ref.yuv"), os.path.join(td, "cur.yuv")
            ref.tofile(rp)
            cur.tofile(cp)
            ms = []
            for _ in range(3):
                r = subprocess.run([mes, cp, rp, td, str(blk), str(span), str(ref.shape[1]),
                                    str(ref.shape[0])], capture_output=True, text=True, timeout=300)
                for line in r.stdout.splitlines():
                    if line.startswith("Computation time:"):
                        ms.append(float(line.split()[2]))
            if ms:
                m = statistics.median(ms)
                out[key] = {
                    "value": cands / (m / 1e3), "unit": "candidates/s", "cores": 100,
                    "kind": "reference", "cost": "mse",
                    "sample": f"unmodified src/cpu (gcc {opt}) on the same frame pair, its own "
                              f"100-thread pool, 'Computation time' median of 3 ({m:.0f} ms)"}
    return out, (field[0] if begin == 0 and end == nbx * nby else None)


def host_stream(eng, w, h, blk, span, cost, seed, sx, sy, frame_ms, batch_frame_ms, cands_frame,
                ramp_ms):
    """Frame-pair streaming from host memory (me_search_pairs):
    a synthetic pan, consecutive pairs, frames uploaded over PCIe inside the
    timed call (pinned: direct DMA; pageable: staged), MV records copied back.
    Reported beside `value`, never as it: `value` has the inputs in HBM."""
    import motionestimation_amd as me
    from motionestimation_amd import synth
    npairs = 64 if w * h <= 2_100_000 else (16 if w * h <= 8_300_000 else 4)
    pinned = me.pinned_frames(npairs + 1, h, w)
    synth.sequence(w, h, npairs + 1, seed, sx, sy, out=pinned)
    pageable = np.array(pinned)
    pairs = [(k, k + 1) for k in range(npairs)]
    out = {"pairs": npairs, "workload": f"{npairs + 1}-frame pan, consecutive pairs"}
    last = {}
    for name, frames in (("pinned", list(pinned)), ("pageable", list(pageable))):
        eng.search_pairs(frames, pairs, blk, span, cost)  # allocates the device slots
        t0 = time.perf_counter()  # clock ramp, as before the other legs (warm())
        while (time.perf_counter() - t0) * 1e3 < ramp_ms:
            eng.search_pairs(frames, pairs, blk, span, cost)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            res = eng.search_pairs(frames, pairs, blk, span, cost)
        dt = (time.perf_counter() - t0) / reps
        last[name] = res
        out[name] = {"pairs_per_s": npairs / dt, "candidates_per_s": cands_frame * npairs / dt,
                     "ms_per_pair": dt / npairs * 1e3}
    # The last timed call's records (both memories) against each pair searched
    # on its own (me_full_search: another entry point, one frame per launch).
    bad = []
    for k, (r, q) in enumerate(pairs):
        smv, sco = eng.full_search(pageable[r], pageable[q], blk, span, cost)
        for name in ("pinned", "pageable"):
            mv, co = last[name]
            if not (np.array_equal(mv[k], smv) and np.array_equal(co[k], sco)):
                bad.append(f"{name} pair {k}")
    out["parity"] = {"ok": not bad, "pairs_checked": npairs, "mismatches": bad[:8],
                     "what": "the last timed call's records (pinned and pageable frames) == "
                             "me_full_search of each pair"}
    # the kernels alone, inputs in HBM: one frame per launch, and per frame of
    # a batched launch
    out["kernel_only_pairs_per_s"] = 1e3 / frame_ms
    out["kernel_only_batched_pairs_per_s"] = 1e3 / batch_frame_ms
    del pinned
    return out


def warm(fn, ms):
    """Untimed calls of fn for `ms` of wall time (synchronising every 4): the
    GPU clock drops during host-side gaps (the parity checks between legs) and
    takes ~25 ms of load to come back (profiles/r03m_clock_ramp.json)."""
    import torch
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()


def single_frame(eng, ref_t, cur_t, blk, span, cost, nb, cands_frame, dev, steps, pins, ramp_ms):
    """One frame per launch on the same resident pair (HIP events on the
    launch stream): what batching saves is launch gaps and per-launch tails.
    The last timed search's field is checked against pins[0] (ref_t is frame 0)."""
    import torch
    h, w = ref_t.shape
    mv = torch.empty((nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(nb, dtype=torch.int32, device=dev)
    warm(lambda: eng.full_search_device(ref_t, cur_t, blk, span, cost, mv, co), ramp_ms)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        eng.full_search_device(ref_t, cur_t, blk, span, cost, mv, co)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    par = verify_fields(eng, batch_fields(mv, co, 1), None, None, w, h, blk, span, cost,
                        pins[:1], dev, singles=False)
    return {"value": cands_frame / (ms / 1e3), "unit": "candidates/s", "kernel_ms": ms,
            "steps": steps, "workload": "one frame per launch (me_full_search_device)",
            "parity": par}


def ssd_beside(eng, ref_t, cur_t, blk, span, nb, cands_frame, dev, steps, pins, ramp_ms, config):
    """The reference's own cost (MSE = SSD / 256) on the step's resident frame
    pairs ([F, H, W] stacks): B = 16 SSD runs on the matrix cores (i8 MFMA), the
    F frames in one batched call (16 1080p frames: one band-walk launch plus
    the lean kernel's launch for the partial bottom block rows).  Reported
    beside `value`; `kernel_ms` is per frame.  roofline.traffic: PMC bytes per
    launch of the dominant kernel from the committed profile of the same
    batch (tools/profile_all.sh, `<config>_b16_s<S>_ssd_f<F>`), and per frame
    over every kernel of the search beside the algorithmic bytes.  The last
    timed batch's fields are checked against the reference's own (pins) and
    single searches."""
    import torch
    F, h, w = ref_t.shape
    nby = (h + blk - 1) // blk
    mv = torch.empty((F * nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(F * nb, dtype=torch.int32, device=dev)
    run = eng.prepared_batch_search(ref_t, 0, cur_t, 0, w, h, blk, span, "ssd", 0, nby, mv, co)
    warm(run, ramp_ms)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps / F
    tops = 2.0 * exact_absdiffs(w, h, blk, span) / (ms / 1e3) / 1e12
    import motionestimation_amd as me
    kernel = me.last_search_path()
    par = verify_fields(eng, batch_fields(mv, co, F), ref_t, cur_t, w, h, blk, span, "ssd",
                        pins, dev)
    traffic, traffic_search = load_traffic(f"{config}_b{blk}_s{span}_ssd_f{F}")
    return {"value": cands_frame / (ms / 1e3), "unit": "candidates/s", "kernel_ms": ms,
            "steps": steps, "frames_per_step": F, "cost": "ssd (reference MSE argmin, bit-exact)",
            "kernel_path": kernel,
            "roofline": {"bound": "mfma", "achieved": tops, "peak": I8_PEAK_TOPS,
                         "unit": "TFLOP/s", "frac": tops / I8_PEAK_TOPS,
                         "traffic": traffic,
                         "traffic_per_frame": traffic_search / F if traffic_search else None,
                         "algorithmic_bytes_per_frame": 2 * w * h + 8 * nb},
            "parity": par}


def ssd_single(eng, ref_t, cur_t, blk, span, nb, cands_frame, dev, steps, pins, ramp_ms, config):
    """The reference's own cost and call shape: ONE 16x16 SSD search per call
    (the drop-in seam me_find_best_blocks / me_full_search replaces
    src/cpu/main.c:144-158 with) on frame 0 of the step, on the path the
    automatic planner picks for a single frame (`kernel_path`).  kernel_ms
    from HIP events on the launch stream over `steps` back-to-back calls;
    roofline against the dense i8 MFMA peak like ssd_mfma, with the PMC
    traffic of the committed one-frame profile (`<config>_b16_s<S>_ssd_f1`,
    tools/profile_all.sh) beside the algorithmic bytes.  The last call's
    field is checked against the unmodified reference's pin of frame 0."""
    import torch
    import motionestimation_amd as me
    h, w = ref_t.shape
    mv = torch.empty((nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(nb, dtype=torch.int32, device=dev)
    run = lambda: eng.full_search_device(ref_t, cur_t, blk, span, "ssd", mv, co)  # noqa: E731
    warm(run, ramp_ms)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    kernel = me.last_search_path()
    par = verify_fields(eng, batch_fields(mv, co, 1), None, None, w, h, blk, span, "ssd",
                        pins[:1], dev, singles=False)
    tops = 2.0 * exact_absdiffs(w, h, blk, span) / (ms / 1e3) / 1e12
    traffic, traffic_search = load_traffic(f"{config}_b{blk}_s{span}_ssd_f1")
    alg = 2 * w * h + 8 * nb
    return {"value": cands_frame / (ms / 1e3), "unit": "candidates/s", "kernel_ms": ms,
            "steps": steps, "kernel_path": kernel,
            "workload": f"{w}x{h} Y, {blk}x{blk}, +-{span}, SSD (reference MSE argmin, bit-exact), "
                        "one frame per call (me_full_search_device)",
            "roofline": {"bound": "mfma", "achieved": tops, "peak": I8_PEAK_TOPS,
                         "unit": "TFLOP/s", "frac": tops / I8_PEAK_TOPS,
                         "traffic": traffic_search if traffic_search else traffic,
                         "algorithmic_bytes": alg,
                         "traffic_over_algorithmic": (traffic_search or traffic) / alg
                         if (traffic_search or traffic) else None},
            "parity": par}


def ssim_beside(eng, ref_t, cur_t, blk, span, nb, dev, steps, ramp_ms):
    """The reference's SSIM search (src/common/ssim.c:44-108, ME_COST_SSIM) on
    frame 0 of the step (the committed golden ssim_synth1080p_b16_s32 is the
    unmodified reference's own field of this pair), one frame per call.

    Roofline.  The reference's per-candidate work is the float cross chain:
    per candidate pixel one exact fma (rounded where the reference's `cv +=`
    rounds) and one subtract, 2 fp32 lane-instructions against the vector
    issue peak (157.3 TFLOPS / 2 flops per fma = 78.6e12 lane-instructions/s);
    `frac` is that reference-equivalent rate (the round-3..5 float kernel ran
    it at 0.74).  Since round 6 the 16 x 16 blocks' cross variance is an exact
    integer computed as an i8 GEMM on the matrix cores (csrc/me_ssim.hip,
    me_ssim_mfma_kernel), so frac > 1 means past that roofline; `mfma` prices
    the GEMM (2 x 256 i8 ops per candidate) against the dense I8 peak.  The
    time covers both launches (statistics, matrix-core search)."""
    import torch
    import motionestimation_amd as me
    sys.path.insert(0, os.path.join(REPO, "tests"))
    h, w = ref_t.shape
    mv = torch.empty((nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(nb, dtype=torch.int32, device=dev)
    run = lambda: eng.full_search_device(ref_t, cur_t, blk, span, "ssim", mv, co)  # noqa: E731
    warm(run, ramp_ms)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    cands = me.candidate_count(w, h, blk, span)
    pix = exact_absdiffs(w, h, blk, span)  # candidate pixels: sum of w*h x candidates
    lane_ops = 2.0 * pix
    peak_lane = 157.3e12 / 2
    tops = 2.0 * pix / (ms / 1e3) / 1e12
    out = {"value": cands / (ms / 1e3), "unit": "candidates/s", "kernel_ms": ms, "steps": steps,
           "workload": f"{w}x{h} Y, {blk}x{blk}, +-{span}, SSIM (reference ssim.c float order, "
                       "bit-exact), one frame per call",
           "roofline": {"bound": "valu_fp32", "model": "reference-equivalent float cross chain",
                        "achieved_lane_instr_per_s": lane_ops / (ms / 1e3),
                        "peak_lane_instr_per_s": peak_lane,
                        "frac": lane_ops / (ms / 1e3) / peak_lane,
                        "flops_frac": 3.0 * pix / (ms / 1e3) / 157.3e12,
                        "mfma": {"achieved": tops, "peak": I8_PEAK_TOPS, "unit": "TOPS",
                                 "frac": tops / I8_PEAK_TOPS},
                        "note": "2 fp32 lane-instructions per candidate pixel (the reference's "
                                "chain); the 16x16 path computes it as an exact-integer i8 GEMM, "
                                "so frac > 1 is past that roofline; both launches timed"}}
    par = {"ok": False, "golden": None}
    try:
        import oracle_lib as O
        man = O.manifest()
        case = [c for c in man["ssim_cases"] if c["width"] == w and c["height"] == h and
                c["blk"] == blk and c["span"] == span]
        if case:
            gmv, gscore = O.load_case(case[0])
            dc = device_check(eng)
            mvh, bits = mv.cpu().numpy(), co.cpu().numpy().view(np.uint32)
            pos = gscore > 0
            eq = bool(np.array_equal(bits, gscore.view(np.uint32)) and
                      np.array_equal(mvh[pos].astype(np.int32), gmv[pos]) and
                      not mvh[~pos].any())
            par = {"ok": eq and dc == "ok", "device_check": dc, "golden": case[0]["name"],
                   "pin_source": "tests/golden: unmodified reference SSIM search (ref_dump_ssim)",
                   "score_bits_equal": bool(np.array_equal(bits, gscore.view(np.uint32)))}
    except (OSError, ValueError, KeyError) as e:  # golden unreadable: reported, leg fails
        par = {"ok": False, "error": str(e)}
    out["parity"] = par
    return out


def batch_frames(ref, cur, nframes):
    """The step's batch: frame 0 is the config's synthetic pair, frame f > 0 the
    same pair with every row rotated by 37 f columns (distinct block contents,
    same statistics; no extra seconds of synthesis per frame at 4K)."""
    return [(ref, cur) if f == 0 else (np.roll(ref, 37 * f, axis=1), np.roll(cur, 37 * f, axis=1))
            for f in range(nframes)]


# ------------------------------------------------------ parity of timed work
def load_pins(cfg_name, blk, span, cost):
    """Per-frame SHA-256 pins of batch_frames(named pair of cfg_name) under this
    search (tests/golden/bench_pins.json, made by tests/golden/make_bench_pins.py:
    SSD from the unmodified reference, SAD from the oracle restatement), or []."""
    try:
        with open(os.path.join(REPO, "tests", "golden", "bench_pins.json")) as f:
            d = json.load(f).get(f"{cfg_name}_b{blk}_s{span}_{cost}")
    except (OSError, ValueError):
        return []
    return list(d["frame_sha256"]) if d else []


def record_stream(mv, cost, w, h, blk, kind):
    """One frame's field in the pinned record format: SAD int16 mvx, int16 mvy,
    uint32 sad; SSD the reference's int32 mvx, int32 mvy, float32 mse with
    mse = (float)SSD / (float)(w*h) of each (edge-clipped) block."""
    mv = np.ascontiguousarray(mv, np.int16).reshape(-1, 2)
    cost = np.ascontiguousarray(cost).view(np.uint32).reshape(-1)
    if kind == "ssd":
        nbx, nby = (w + blk - 1) // blk, (h + blk - 1) // blk
        bw = np.minimum(blk, w - np.arange(nbx) * blk)
        bh = np.minimum(blk, h - np.arange(nby) * blk)
        area = (bh[:, None] * bw[None, :]).reshape(-1).astype(np.float32)
        rec = np.empty((len(mv), 3), np.int32)
        rec[:, :2] = mv
        rec[:, 2] = (cost.astype(np.float32) / area).view(np.int32)
        return rec.tobytes()
    rec = np.empty((len(mv), 8), np.uint8)
    rec[:, :4] = mv.view(np.uint8).reshape(-1, 4)
    rec[:, 4:] = cost.view(np.uint8).reshape(-1, 4)
    return rec.tobytes()


def pin_matches(fields, pins, w, h, blk, kind):
    """Frames of `fields` ([(mv, cost)] in batch order) equal to their pins:
    (checked, equal)."""
    import hashlib
    n = min(len(fields), len(pins))
    eq = sum(hashlib.sha256(record_stream(mv, co, w, h, blk, kind)).hexdigest() == pins[f]
             for f, (mv, co) in enumerate(fields[:n]))
    return n, eq


def device_check(eng):
    """me_device_check after the stream drained: 'ok' or the library's error."""
    import torch
    from motionestimation_amd import MEError
    torch.cuda.synchronize()
    try:
        eng.device_check()
        return "ok"
    except MEError as e:
        return str(e)


def batch_fields(mv_t, cost_t, F):
    """[(mv int16 [nb, 2], cost uint32 [nb])] per frame of a batched search's outputs."""
    mv = mv_t.cpu().numpy().reshape(F, -1, 2)
    co = cost_t.cpu().numpy().view(np.uint32).reshape(F, -1)
    return [(mv[f], co[f]) for f in range(F)]


def verify_fields(eng, fields, ref_t, cur_t, w, h, blk, span, cost, pins, dev, singles=True):
    """Parity of a timed step's fields (frame f of the batch = ref_t[f], cur_t[f]):
    me_device_check clean; each frame equal to a one-frame-per-call search
    (me_full_search_device: a different launch shape on the same planes); each
    frame with a pin equal to it (pins: SSD the unmodified reference, SAD the
    oracle restatement).  Returns the record with "ok"."""
    import torch
    out = {"device_check": device_check(eng), "frames": len(fields)}
    ok = out["device_check"] == "ok"
    if singles and ref_t is not None:
        nb = len(fields[0][0])
        smv = torch.empty((nb, 2), dtype=torch.int16, device=dev)
        sco = torch.empty(nb, dtype=torch.int32, device=dev)
        same = 0
        for f, (mv, co) in enumerate(fields):
            smv.fill_(-1)
            eng.full_search_device(ref_t[f], cur_t[f], blk, span, cost, smv, sco)
            torch.cuda.synchronize()
            same += bool(np.array_equal(smv.cpu().numpy(), mv) and
                         np.array_equal(sco.cpu().numpy().view(np.uint32), co))
        out["single_frame_equal"] = same
        dc = device_check(eng)
        ok = ok and same == len(fields) and dc == "ok"
        if dc != "ok":
            out["device_check"] = dc
    n, eq = pin_matches(fields, pins, w, h, blk, cost)
    out["pinned_frames"], out["pinned_equal"] = n, eq
    out["pin_source"] = ("tests/golden/bench_pins.json: " +
                         ("unmodified reference (ref_dump)" if cost == "ssd" else
                          "oracle/me_oracle.c restatement")) if n else None
    out["ok"] = bool(ok and eq == n)
    return out


class StripeRun:
    """F frames per step in row stripes over the ranks.

    Rank r holds, for each of the step's F frames, one stripe's cur rows and
    ref rows with the S-row halo, searches all F stripes together
    (me_search_stripes_device: one launch where the kernels allow), and sends
    its padded records to rank 0 in one gather per step.  With RCCL the gather is the library's ncclGather,
    enqueued right after the search on the same stream: the host never waits
    inside the timed region."""

    def __init__(self, eng, dev, world, rank, gloo, frames, blk, span, cost, graph=False,
                 comm_timeout_ms=60000):
        import torch
        import torch.distributed as dist
        from motionestimation_amd import shard
        h, w = frames[0][0].shape
        F = len(frames)
        self.eng, self.dev, self.world, self.rank, self.gloo = eng, dev, world, rank, gloo
        self.w, self.h, self.blk, self.span, self.cost, self.nframes = w, h, blk, span, cost, F
        self.comm_timeout_ms = comm_timeout_ms
        self.stripes = shard.plan(w, h, blk, span, world)
        # Rank r searches stripe (r + f) % N of frame f: over N frames every
        # rank holds every stripe once, so the ranks' rows balance exactly
        # (an 8-way 1080p split has 9- and 8-row stripes: 9-row ranks took
        # 92.8 us per 8 frames against 78.5, profiles/r03o_*).
        self.own = [self.stripes[(rank + f) % world] for f in range(F)]
        self.st = self.own[0]
        mb = self.stripes[0].max_blocks
        ref_rows = max(st.ref_y1 - st.ref_y0 for st in self.own)
        cur_rows = max(st.cur_y1 - st.cur_y0 for st in self.own)
        self.ref_t = torch.zeros((F, ref_rows, w), dtype=torch.uint8, device=dev)
        self.cur_t = torch.zeros((F, cur_rows, w), dtype=torch.uint8, device=dev)
        for f, ((r, c), st) in enumerate(zip(frames, self.own)):
            self.ref_t[f, :st.ref_y1 - st.ref_y0] = torch.from_numpy(r[st.ref_y0:st.ref_y1].copy())
            self.cur_t[f, :st.cur_y1 - st.cur_y0] = torch.from_numpy(c[st.cur_y0:st.cur_y1].copy())
        # records: frame f's stripe at [f * max_blocks, f * max_blocks + its nblocks)
        self.recs = [torch.zeros((2, F * mb), dtype=torch.int32, device=dev) for _ in range(2)]
        self.mb = mb
        cdev = torch.device("cpu") if gloo else dev
        self.i = 0
        # RCCL ranks gather in libme_hip (me_gather_device) on the search's own
        # stream, through calls marshalled once: a small stripe's step is bound
        # by host time.  torch.distributed.gather cost ~30 us of host time per
        # call, and a side stream's event handshake ~15 us more than it saves
        # (the persistent search kernel holds every CU, so the gather cannot run
        # beside it): 8-way 1080p stripe step 36-49 us -> 21-24 us on one GPU
        # (profiles/r02au_step_overhead.jsonl ... r02ax_step_overhead_prepared.jsonl).
        # (a one-rank RCCL group under torch.distributed.run takes this path too:
        # the GPU test of the library gather on a one-GPU box)
        self.lib = dist.is_initialized() and not gloo
        mvs = [r[0].view(torch.int16).view(F * mb, 2) for r in self.recs]
        jobs = [[(self.ref_t[f], st.ref_y0, self.cur_t[f], st.cur_y0, st.row_begin, st.row_end,
                  mvs[k][f * mb:], self.recs[k][1][f * mb:])
                 for f, st in enumerate(self.own) if st.nblocks] for k in range(2)]
        self.run_search = [eng.prepared_stripes_search(w, h, blk, span, cost, jobs[k], stride=w)
                           if jobs[k] else (lambda: None) for k in range(2)]
        self.graphs = None
        if self.lib:
            if not eng.comm_ranks:  # one communicator per context (stripe_4k reuses it)
                uid = torch.zeros(128, dtype=torch.uint8,  # host tensor on the gloo control plane
                                  device=dev if dist.get_backend() == "nccl" else "cpu")
                if rank == 0:
                    uid.copy_(torch.frombuffer(bytearray(eng.comm_unique_id()), dtype=torch.uint8))
                dist.broadcast(uid, 0)
                eng.comm_init(bytes(uid.cpu().numpy().tobytes()), world, rank)
            self.flat = [torch.empty((world,) + tuple(r.shape), dtype=r.dtype, device=dev)
                         if rank == 0 else None for r in self.recs]
            self.bufs = [list(f) if f is not None else None for f in self.flat]
            self.run_gather = [eng.prepared_gather(self.recs[k], self.flat[k]) for k in range(2)]
            # --graph: one hipGraph per record buffer holding the search and its
            # gather (me_capture_begin/end), one graph launch per step.  Not the
            # default: on one GPU a replay cost more than the two direct
            # enqueues (8-way 1080p stripe step 24.6 vs 22.0 us, search alone
            # 20.6 vs 15.5 us; hipGraphLaunch's host time, profiles/r03a_step_overhead_graph.jsonl).
            # Each is run once uncaptured first: that sizes the search scratch
            # and sets up RCCL's connections.
            if graph and jobs[0]:
                from motionestimation_amd import MEError
                stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
                for k in range(2):
                    self.run_search[k]()
                    self.run_gather[k]()
                self.drain()
                torch.cuda.synchronize()
                try:
                    self.graphs = [eng.capture(stream, lambda k=k: (self.run_search[k](),
                                                                     self.run_gather[k]()))
                                   for k in range(2)]
                    self.run_graph = [g.prepared(stream) for g in self.graphs]
                except MEError as e:  # reported in the line (config.gather)
                    print(f"bench.py: graph capture failed, direct enqueue: {e}", file=sys.stderr)
                    self.graphs = None
        else:
            self.bufs = [[torch.empty_like(r, device=cdev) for _ in range(world)] if rank == 0
                         else None for r in self.recs]

    def step(self):
        import torch.distributed as dist
        k = self.i & 1
        self.i += 1
        if self.lib:  # search, then the one exchange, in stream order (no host sync)
            if self.graphs:
                self.run_graph[k]()
                return k
            self.run_search[k]()
            self.run_gather[k]()
            return k
        self.run_search[k]()
        if self.world > 1:  # gloo rehearsal: per-stripe MV records -> rank 0
            dist.gather(self.recs[k].cpu(), self.bufs[k], dst=0)
        return k

    def drain(self):
        """Bounded wait for this rank's searches and gathers (RCCL ranks):
        me_comm_check raises ME_ECOMM (and aborts the communicator, so the
        stream can drain) when a peer stalled or died, instead of the next
        synchronize blocking until the driver's timeout."""
        if self.lib:
            self.eng.comm_check(self.comm_timeout_ms)

    def gather_impl(self):
        if self.world == 1 and not self.lib:
            return None
        if not self.lib:
            return "torch.distributed.gather (gloo rehearsal)"
        return ("me_gather_device (RCCL ncclGather in libme_hip, on the search stream)" +
                (", search + gather captured in one hipGraph per record buffer"
                 if self.graphs else ""))

    def gathered_fields(self):
        """A last, synchronous step; rank 0 returns [(mv, cost)] per frame."""
        import torch
        from motionestimation_amd import shard
        k = self.step()
        self.drain()
        torch.cuda.synchronize()
        if self.rank != 0:
            return None
        recs = [self.recs[k].cpu()] if self.world == 1 and not self.lib else self.bufs[k]
        recs = [np.asarray(r.cpu() if hasattr(r, "cpu") else r) for r in recs]
        out = []
        for f in range(self.nframes):
            # stripe s of frame f: rank (s - f) mod N, record slot f
            per_stripe = [recs[(s - f) % self.world][:, f * self.mb:f * self.mb + st.nblocks]
                          for s, st in enumerate(self.stripes)]
            out.append(shard.assemble(per_stripe, self.stripes))
        return out


def clock_ramp(step, ms, world, drain=None):
    """Untimed steps until `ms` of wall time has passed on every rank (ranks
    agree through a MIN all-reduce, so a collective inside the step runs the
    same number of times everywhere).  The GPU's clock ramps up under load:
    back-to-back 1080p searches run 76 -> 69 us over the first ~25 ms, and again
    after 1 s idle (tools/dbg/ramp_probe.py, profiles/r03m_clock_ramp.json).
    Returns the steps run."""
    import torch
    import torch.distributed as dist
    t0, n = time.perf_counter(), 0
    while ms > 0:
        for _ in range(4):
            step()
        n += 4
        (drain or torch.cuda.synchronize)()
        el = time.perf_counter() - t0
        if world > 1:
            gloo = dist.get_backend() == "gloo"
            t = torch.tensor([el], dtype=torch.float64,
                             device="cpu" if gloo else torch.device("cuda", torch.cuda.current_device()))
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            el = float(t[0])
        if el * 1e3 >= ms:
            break
    return n


def timed(step, steps, warmup, world, finish=None, ramp_ms=0, drain=None):
    """The clock ramp (clock_ramp), W untimed steps, then K steps between
    barrier + synchronize; returns (max-over-ranks wall seconds, max-over-ranks
    ms per step on the current stream from one HIP event pair around the region).
    drain: a bounded wait for the stream run before each synchronize (RCCL
    ranks: me_comm_check, which raises ME_ECOMM instead of hanging when a peer
    rank stalled or died)."""
    import torch
    import torch.distributed as dist
    drain = drain or (lambda: None)
    clock_ramp(step, ramp_ms, world, lambda: (drain(), torch.cuda.synchronize()))
    for _ in range(warmup):
        step()
    if finish:
        finish()
    drain()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        step()
    if finish:
        finish()
    ev1.record()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps
    if world > 1:
        gloo = dist.get_backend() == "gloo"
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64,
                         device="cpu" if gloo else torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def all_ranks_ok(ok, world):
    """True on every rank iff `ok` is true on every rank (MIN all-reduce)."""
    if world == 1:
        return bool(ok)
    import torch
    import torch.distributed as dist
    gloo = dist.get_backend() == "gloo"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                     device="cpu" if gloo else torch.device("cuda", torch.cuda.current_device()))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t[0]))


def stripe_parity(eng, sr, frames, dev, pins):
    """Parity of a stripe run's last step (not timed).  Every rank: its
    searches' me_device_check is clean.  Rank 0: the gathered stripe fields of
    every frame of the step equal one batched full-frame search on one GPU and
    their pins (frame f of the step = batch_frames' frame f).  Returns the
    record on rank 0 ({"ok"} elsewhere); "ok" covers every rank."""
    import torch
    import motionestimation_amd as me
    fields = sr.gathered_fields()
    dc = device_check(eng)
    rec = None
    if sr.rank == 0:
        h, w = frames[0][0].shape
        nb = me.num_blocks(w, h, sr.blk)
        F = len(frames)
        fmv = torch.empty((F * nb, 2), dtype=torch.int16, device=dev)
        fco = torch.empty(F * nb, dtype=torch.int32, device=dev)
        eng.search_batch_device(torch.from_numpy(np.stack([r for r, _ in frames])).to(dev), 0,
                                torch.from_numpy(np.stack([c for _, c in frames])).to(dev), 0, w,
                                h, sr.blk, sr.span, sr.cost, 0, (h + sr.blk - 1) // sr.blk, fmv,
                                fco)
        torch.cuda.synchronize()
        batch = batch_fields(fmv, fco, F)
        same = sum(bool(np.array_equal(g[0], b[0]) and np.array_equal(g[1], b[1]))
                   for g, b in zip(fields, batch))
        n, eq = pin_matches(fields, pins, w, h, sr.blk, sr.cost)
        rec = {"frames": F, "batched_equal": same, "pinned_frames": n, "pinned_equal": eq,
               "pin_source": "tests/golden/bench_pins.json" if n else None}
        ok = dc == "ok" and same == F and eq == n
    else:
        ok = dc == "ok"
    ok = all_ranks_ok(ok, sr.world)
    if rec is not None:
        rec["device_check"] = dc if sr.world == 1 else ("ok on every rank" if ok else
                                                        f"rank 0: {dc} (see every rank's stderr)")
    if dc != "ok":
        print(f"bench.py: rank {sr.rank}: {dc}", file=sys.stderr)
    rec = rec if rec is not None else {}
    rec["ok"] = ok
    return rec


def stripe_record(eng, dev, world, rank, gloo, cfg_name, cost, steps, warmup, nframes,
                  graph=False, ramp_ms=0, comm_timeout_ms=60000):
    """Nested record: a BASELINE config in stripe mode on the same ranks."""
    import motionestimation_amd as me
    from motionestimation_amd import synth
    cfg, blk, span = CONFIGS[cfg_name]
    w, h, seed, sx, sy = synth.CONFIGS[cfg]
    frames = batch_frames(*synth.frame_pair(w, h, seed, sx, sy), nframes)
    cands = me.candidate_count(w, h, blk, span)
    sr = StripeRun(eng, dev, world, rank, gloo, frames, blk, span, cost, graph, comm_timeout_ms)
    elapsed, kern_ms = timed(sr.step, steps, warmup, world, ramp_ms=ramp_ms, drain=sr.drain)
    parity = stripe_parity(eng, sr, frames, dev, load_pins(cfg_name, blk, span, cost))
    return {"value": cands * nframes * steps / elapsed, "unit": "candidates/s",
            "frames_per_s": nframes * steps / elapsed, "ms_per_step": elapsed / steps * 1e3,
            "kernel_ms": kern_ms, "steps": steps, "warmup": warmup, "n_gpus": world,
            "frames_per_step": nframes, "scaling": "strong", "parallelism": f"stripe{world}",
            "workload": f"{w}x{h} Y, {blk}x{blk} blocks, full search +-{span}, {cost.upper()}, "
                        f"{nframes} frames per step, each in row stripes over the ranks; one "
                        "batched search and one RCCL gather per step",
            "candidates_per_frame": cands,
            "stripe_gather_parity": parity["ok"] if parity else None, "parity": parity,
            "gather": sr.gather_impl()}


def sad_frames_per_launch(w, h, blk, span, F):
    """Frames per SAD launch of an F-frame batch: one launch of up to MAX_JOBS
    frames (me_kernels.hip launch_flow_jobs / launch_item_jobs), 8K included."""
    return min(F, MAX_JOBS)


def ssd_frames_per_launch(w, h, blk, span, F):
    """Frames per matrix-core launch pair of an F-frame SSD batch (me_mfma.hip
    launch_mfma_jobs): B = 16 (block-major kernel, S <= 192) batches as many
    frames as MAX_JOBS and 1 GiB of prepass planes allow (rp plane + one or two
    4-byte S2 planes over the rows + 16, 256-byte aligned); 8x8 searches
    launch per frame."""
    if blk != 16 or span > 192 or F < 2:
        return 1
    rows = h + 16  # whole frames: resident rows 0..H (ya0 = 0)
    plane = rows * ((w + 15) & ~15)
    r256 = lambda v: (v + 255) & ~255  # noqa: E731
    stride = r256(r256(plane) + (2 if h % 16 else 1) * 4 * plane)
    m = min(MAX_JOBS, (1 << 30) // stride)
    return min(F, m) if m >= 2 else 1


def load_traffic(tag):
    """(HBM bytes per launch of the dominant kernel, per search over all its
    kernels) from the committed rocprofv3 PMC summary of this workload
    (tools/profile.sh), or (None, None)."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f).get(tag, {})
        return d.get("hbm_bytes_per_launch"), d.get("hbm_bytes_per_search")
    except (OSError, ValueError):
        return None, None


def load_valu(tag):
    """Wave-level instruction counts per batch launch of the dominant kernel
    (SQ_INSTS_VALU incl. MFMA, SQ_INSTS_MFMA) from the committed PMC summary
    (tools/profile.sh VALU=1), or None."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f).get(tag, {})
        k = d.get("kernels", {}).get(d.get("dominant_kernel"), {})
        if "SQ_INSTS_VALU" not in k:
            return None
        return {"kernel": d["dominant_kernel"].split("(")[0], "valu": k["SQ_INSTS_VALU"],
                "mfma": k.get("SQ_INSTS_MFMA"), "profile_tag": d.get("profile_tag")}
    except (OSError, ValueError, KeyError):
        return None


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) with no launcher: start N ranks, one process
    per GPU, as a child `torch.distributed.run` and forward rank 0's JSON line.

    Runs before anything touches the GPU (torch.cuda.device_count() does not
    initialise it on this image), so the parent never holds a device while its
    child runs.  Refuses, with a non-zero exit and no JSON line, a request for
    more RCCL ranks than visible devices (gloo ranks may share one GPU: the
    rehearsal mode)."""
    import torch
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {ndev}",
              file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    r = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    for l in r.stdout.splitlines():
        if not l.startswith("{"):
            print(l, file=sys.stderr)
    if r.returncode != 0 or len(lines) != 1:
        print(f"bench.py: {args.gpus}-rank child exited {r.returncode} with {len(lines)} JSON "
              "lines", file=sys.stderr)
        return r.returncode or 3
    d = json.loads(lines[0])
    if d.get("n_gpus") != args.gpus:
        print(f"bench.py: child reported n_gpus {d.get('n_gpus')}", file=sys.stderr)
        return 3
    print(lines[0], flush=True)
    return 0


T_START = time.perf_counter()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    # stdout carries exactly the one JSON line: anything else written to fd 1
    # (RCCL's version banner at communicator init, library messages) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    ndev = torch.cuda.device_count()
    gloo = args.dist_backend == "gloo"
    if ndev < 1 or (not gloo and ndev < world):
        raise SystemExit(f"{world} RCCL ranks need {world} visible GPUs, found {ndev}")
    gpu = local % ndev  # ranks > devices only in a gloo rehearsal on one GPU
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    # Every search of the run goes on one created stream (graph capture needs
    # one; the legacy NULL stream cannot be captured), and the HIP events that
    # time the kernels are recorded on it (torch's current stream).
    torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    # a process group whenever torch.distributed.run launched us (WORLD_SIZE set),
    # a one-rank group included
    launched = "WORLD_SIZE" in os.environ
    if launched:
        # torch's own collectives (barriers, the ramp's MIN, the result MAX)
        # fail after this instead of the default 10 minutes
        import datetime
        tmo = datetime.timedelta(seconds=max(60, 3 * args.comm_timeout_ms // 1000))
        # torch's process group is the control plane only (the id broadcast,
        # barriers, the ramp's MIN and the result's MAX, on host tensors): gloo
        # in both modes.  The one data exchange of an RCCL run is the library's
        # ncclGather (me_gather_device), so a rank holds ONE RCCL communicator
        # and its streams: with torch's "nccl" group as well, a rank held two
        # communicators on top of torch's stream and the search stream, more
        # streams than GPU_MAX_HW_QUEUES = 4.
        if args.torch_pg == "nccl" and not gloo:  # A/B only: the round-4 configuration
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group("gloo", timeout=tmo)

    import motionestimation_amd as me
    from motionestimation_amd import synth

    cfg, blk, span = CONFIGS[args.config]
    w, h, seed, sx, sy = synth.CONFIGS[cfg]
    cands_frame = me.candidate_count(w, h, blk, span)
    nb = me.num_blocks(w, h, blk)
    eng = me.Engine(devices=[gpu])

    mode = args.mode if args.mode != "auto" else ("frames" if world == 1 else "stripe")
    F = args.frames_per_step
    parity = None
    pins = load_pins(args.config, blk, span, args.cost)
    if mode == "frames":
        # rank r: its own batch of F frame pairs (same size; seed varies), all F
        # searched in one launch per step (me_full_search_batch_device)
        ref, cur = synth.frame_pair(w, h, seed + rank, sx, sy)
        frames = batch_frames(ref, cur, F)
        ref_t = torch.from_numpy(np.stack([r for r, _ in frames])).to(dev)
        cur_t = torch.from_numpy(np.stack([c for _, c in frames])).to(dev)
        mv_t = torch.empty((F * nb, 2), dtype=torch.int16, device=dev)
        cost_t = torch.empty(F * nb, dtype=torch.int32, device=dev)
        step = eng.prepared_batch_search(ref_t, 0, cur_t, 0, w, h, blk, span, args.cost, 0,
                                         (h + blk - 1) // blk, mv_t, cost_t)
        units_per_step = cands_frame * F * world
        # Kernel duration: one HIP event pair on the stream the search is
        # launched on (torch's current stream) around the whole timed region,
        # / K (per-step event pairs would stretch the back-to-back launches).
        t_timed = time.perf_counter()
        elapsed, kern_ms = timed(step, args.steps, args.warmup, world, ramp_ms=args.ramp_ms)
        t_verify = time.perf_counter()
        # The timed step's own output (mv_t / cost_t hold the last step's
        # fields): device check, one-frame-per-call searches, and the pins of
        # this batch (rank 0: its frames are the pinned batch_frames).
        parity = verify_fields(eng, batch_fields(mv_t, cost_t, F), ref_t, cur_t, w, h, blk, span,
                               args.cost, pins if rank == 0 else [], dev)
        parity["ok"] = all_ranks_ok(parity["ok"], world)
        t_done = time.perf_counter()
    else:
        t_timed = time.perf_counter()
        ref, cur = synth.frame_pair(w, h, seed, sx, sy)
        frames = batch_frames(ref, cur, F)
        sr = StripeRun(eng, dev, world, rank, gloo, frames, blk, span, args.cost, args.graph,
                       args.comm_timeout_ms)
        units_per_step = cands_frame * F
        elapsed, kern_ms = timed(sr.step, args.steps, args.warmup, world, ramp_ms=args.ramp_ms,
                                 drain=sr.drain)
        t_verify = time.perf_counter()
        parity = stripe_parity(eng, sr, frames, dev, pins)
        t_done = time.perf_counter()

    value = units_per_step * args.steps / elapsed
    # Roofline of the dominant kernel: algorithmic HBM bytes per
    # launch = 2*W*H (u8 ref + cur, read once) + 8*nblocks (mv + cost written)
    # for the planes that launch covers.
    # VALU work: the exact abs-diff count (w*h of each block, not B*B).
    # Stripe mode: the frame's work / N against the slowest rank's kernel time.
    # Priced per launch of the dominant kernel.  SAD batches share launches of
    # up to MAX_JOBS (32) frames (1080p: the flow kernel's job table; 4K: the
    # item kernel's, sad_frames_per_launch); B = 16 SSD batches share a prepass and a block-major
    # launch (ssd_frames_per_launch), 8x8 SSD launches per frame.
    # So a launch holds fpl frames and lasts kern_ms * fpl / F.  Stripe mode:
    # the rank's F stripes, one launch per step (F <= 32).  roofline.traffic is
    # the PMC bytes per launch of the same workload at the same F
    # (tools/profile_all.sh -> profiles/pmc_summary.json).
    fpl = (sad_frames_per_launch(w, h, blk, span, F) if args.cost == "sad"
           else ssd_frames_per_launch(w, h, blk, span, F))
    if mode == "frames":
        alg_bytes = fpl * (2 * w * h + 8 * nb)
        launch_ms = kern_ms * fpl / F
        absdiffs = F * exact_absdiffs(w, h, blk, span)
    else:
        alg_bytes = sum((o.ref_y1 - o.ref_y0 + o.cur_y1 - o.cur_y0) * w + 8 * o.nblocks
                        for o in sr.own)
        launch_ms = kern_ms
        absdiffs = F * exact_absdiffs(w, h, blk, span) / world
    achieved = alg_bytes / (launch_ms / 1e3) / 1e9
    tag = f"{args.config}_b{blk}_s{span}_{args.cost}_f{F}"
    traffic, traffic_search = load_traffic(tag) if mode == "frames" else (None, None)
    line = {
        "metric": METRIC if args.config == "1080p" and args.cost == "sad" else
        f"{blk}x{blk} {args.cost.upper()} candidates/sec at {args.config} +-{span}",
        "value": value,
        "unit": "candidates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "clock_ramp_ms": args.ramp_ms,
        "higher_is_better": True,
        "scaling": "weak" if mode == "frames" else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic: motionestimation_amd.synth '{cfg}' (splitmix64 seed {seed}"
                f"{'+rank' if mode == 'frames' and world > 1 else ''}, 5x5 box, cur = ref shifted "
                f"({sx:+d},{sy:+d}) + uniform [-2,2])",
        "config": {"workload": f"{w}x{h} Y, {blk}x{blk} blocks, full search +-{span}, "
                               f"{args.cost.upper()}, " +
                               (f"{F} frame pairs per rank per step in one batched search"
                                if mode == "frames" else
                                f"{F} frames per step, each in row stripes over the ranks; one "
                                "batched search and one RCCL gather per step"),
                   "width": w, "height": h, "block": blk, "range": span, "cost": args.cost,
                   "candidates_per_frame": cands_frame, "blocks_per_frame": nb,
                   "frames_per_step": F, "parallelism": f"{mode}{world}"},
        "kernel_ms": kern_ms,
        "kernel_ms_per_unit": launch_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_per_search": traffic_search,
                     "algorithmic_bytes": alg_bytes,
                     "per": "launch" if mode == "frames" else "rank step",
                     "frames_per_launch": fpl if mode == "frames" else F,
                     "launch_ms": launch_ms,
                     "valu": {"achieved_absdiff_per_s": absdiffs / (kern_ms / 1e3),
                              "peak_absdiff_per_s": VALU_PEAK_ABSDIFF,
                              "frac": absdiffs / (kern_ms / 1e3) / VALU_PEAK_ABSDIFF}},
        "cpu_baseline": None,
    }
    if args.cost == "ssim":  # float chains, not abs-diffs: no VALU-peak claim
        line["roofline"]["valu"] = None
    if args.cost == "ssd" and blk in (8, 16):
        # B = 8 and 16 SSD run on the matrix cores (i8 MFMA cross term): the bound is
        # the MFMA peak; algorithmic ops = 2 x B*B multiply-adds per candidate
        ops = 2.0 * absdiffs
        tops = ops / (kern_ms / 1e3) / 1e12
        hbm = line["roofline"]
        hbm.pop("valu", None)
        line["roofline"] = {"bound": "mfma", "achieved": tops, "peak": I8_PEAK_TOPS,
                            "unit": "TFLOP/s", "frac": tops / I8_PEAK_TOPS, "traffic": traffic,
                            "traffic_per_search": traffic_search,
                            "note": "useful int8 ops (2*w*h per candidate) over the whole search "
                                    "(S2 prepass + MFMA kernel); dense i8 peak",
                            "hbm": {k: hbm[k] for k in ("achieved", "peak", "unit", "frac",
                                                        "algorithmic_bytes", "per",
                                                        "frames_per_launch", "launch_ms")}}
        vc = load_valu(tag) if blk == 8 and mode == "frames" else None
        if vc:
            # 8x8: the MFMA does a quarter of a 16x16 block's work per candidate
            # and the per-candidate key build + min is VALU, the real bound
            # (VERDICT r5 #3): the kernel's non-MFMA VALU lane-instructions per
            # launch (rocprofv3 SQ_INSTS_VALU - SQ_INSTS_MFMA, x 64 lanes) over
            # this run's launch time, against the vector issue peak (256 CUs x 4
            # SIMD-32 x 2.4 GHz: one wave64 instruction per 2 clocks per SIMD)
            lane = 64.0 * (vc["valu"] - (vc["mfma"] or 0.0))
            cands_launch = cands_frame * fpl
            line["roofline"]["valu"] = {
                "kernel": vc["kernel"], "profile_tag": vc["profile_tag"],
                "lane_instr_per_launch": lane, "lane_instr_per_candidate": lane / cands_launch,
                "achieved_lane_instr_per_s": lane / (launch_ms / 1e3),
                "peak_lane_instr_per_s": VALU_PEAK_LANE,
                "frac": lane / (launch_ms / 1e3) / VALU_PEAK_LANE}
    # Parity of every measured leg: the line verifies the work
    # its own timed regions did; `parity` is false and the exit status
    # non-zero if any leg's fields differ or a kernel reported ME_EDEVICE.
    legs = {"timed_step": parity}
    # wall seconds of every leg (stderr and the line's `wall_s`): what the
    # driver's clock around this command covers besides the timed region
    wall = {"startup": t_timed - T_START, "timed_step (warmup, ramp, K steps)": t_verify - t_timed,
            "timed_step_parity": t_done - t_verify}

    def leg_clock(name, t0):
        wall[name] = time.perf_counter() - t0
        print(f"bench.py: leg {name}: {wall[name]:.2f} s", file=sys.stderr, flush=True)
    if mode == "stripe":
        line["stripe_gather_parity"] = parity.get("batched_equal") == F if rank == 0 else None
        line["config"]["gather"] = sr.gather_impl()
    if rank == 0 and world == 1 and mode == "frames" and F > 1 and not args.no_single:
        # the same search one frame per launch (me_full_search_device), for
        # comparison: the batch's only difference is launches per frame
        t0 = time.perf_counter()
        line["single_frame"] = single_frame(eng, ref_t[0], cur_t[0], blk, span, args.cost, nb,
                                            cands_frame, dev, min(args.steps * F, 100), pins,
                                            args.ramp_ms)
        legs["single_frame"] = line["single_frame"]["parity"]
        leg_clock("single_frame", t0)
    if (rank == 0 and world == 1 and mode == "frames" and args.cost == "sad"
            and blk == 16 and not args.no_ssd):
        t0 = time.perf_counter()
        ssd_pins = load_pins(args.config, blk, span, "ssd")
        line["ssd_mfma"] = ssd_beside(eng, ref_t, cur_t, blk, span, nb, cands_frame, dev,
                                      min(args.steps, 20), ssd_pins, args.ramp_ms, args.config)
        legs["ssd_mfma"] = line["ssd_mfma"]["parity"]
        leg_clock("ssd_mfma", t0)
        t0 = time.perf_counter()
        line["ssd_single_frame"] = ssd_single(eng, ref_t[0], cur_t[0], blk, span, nb, cands_frame,
                                              dev, min(args.steps * F, 100), ssd_pins,
                                              args.ramp_ms, args.config)
        legs["ssd_single_frame"] = line["ssd_single_frame"]["parity"]
        leg_clock("ssd_single_frame", t0)
    if (rank == 0 and world == 1 and mode == "frames" and args.config == "1080p"
            and args.cost == "sad" and not args.no_ssim):
        t0 = time.perf_counter()
        line["ssim"] = ssim_beside(eng, ref_t[0], cur_t[0], blk, span, nb, dev,
                                   min(args.steps, 10), args.ramp_ms)
        legs["ssim"] = line["ssim"]["parity"]
        leg_clock("ssim", t0)
    if rank == 0 and world == 1 and not args.no_cpu:
        t0 = time.perf_counter()
        line["cpu_baseline"], field = cpu_baselines(ref, cur, blk, span, args.cost,
                                                    args.cpu_threads, cands_frame)
        leg_clock("cpu_baseline", t0)
        if field is not None and mode == "frames":
            # the oracle's field of the CPU leg, run live on this box, against
            # frame 0 of the timed step (frame 0 = this ref/cur pair)
            mv0, co0 = batch_fields(mv_t, cost_t, F)[0]
            eq = bool(np.array_equal(field[0], mv0) and np.array_equal(field[1], co0))
            legs["oracle_frame0"] = {"ok": eq, "what": "cpu_baseline's oracle field of frame 0 "
                                                       "== the timed step's frame 0"}
    if not args.no_4k and args.cost in ("sad", "ssd"):
        # BASELINE configs[3] (4K +-64), the config north_star's 8-GPU split is
        # quoted on, in stripe mode on the same ranks (at N = 1: the denominator)
        t0 = time.perf_counter()
        rec4k = stripe_record(eng, dev, world, rank, gloo, "4k", args.cost,
                              min(args.steps, 20), min(args.warmup, 3), F, args.graph,
                              min(args.ramp_ms, 30.0), args.comm_timeout_ms)
        legs["stripe_4k"] = rec4k["parity"]
        leg_clock("stripe_4k", t0)
        if rank == 0:
            line["stripe_4k"] = rec4k
    if rank == 0 and world == 1 and mode == "frames" and not args.no_stream:
        # per-frame kernel times (launch_ms covers a whole batched launch)
        one = line.get("single_frame", {}).get("kernel_ms", kern_ms / F)
        t0 = time.perf_counter()
        line["host_stream"] = host_stream(eng, w, h, blk, span, args.cost, seed, sx, sy,
                                          one, kern_ms / F, cands_frame, args.ramp_ms)
        legs["host_stream"] = line["host_stream"]["parity"]
        leg_clock("host_stream", t0)
    ok = all(leg["ok"] for leg in legs.values())
    line["parity"] = ok
    line["parity_legs"] = legs
    wall["total"] = time.perf_counter() - T_START
    line["wall_s"] = {k: round(v, 3) for k, v in wall.items()}
    print(f"bench.py: wall {json.dumps(line['wall_s'])}", file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps(line), file=json_out, flush=True)
    eng.close()
    if launched:
        dist.destroy_process_group()
    if not ok:
        bad = [k for k, leg in legs.items() if not leg["ok"]]
        print(f"bench.py: rank {rank}: parity FAILED in {bad}: {json.dumps(legs)}",
              file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
