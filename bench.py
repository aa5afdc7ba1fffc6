#!/usr/bin/env python3
"""bench.py -- full-search block matching throughput on MI355X.

Metric (BASELINE.json): 16x16 SAD candidates/sec at 1080p +-32; achieved HBM
GB/s vs roofline.  One step = one full search of a 1920x1080 Y-frame pair
(B=16, S=32, SAD, 33,188,832 exact candidates) per rank, inputs resident in
HBM before the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode frames|stripe]
                  [--config 1080p|4k|8k] [--cost sad|ssd] [--no-cpu]

--mode frames (default): each rank searches its own frame pair per step (a
  sequence sharded across GPUs): weak scaling, no collective in the data path.
--mode stripe: ONE frame per step split into candidate-balanced block-row
  stripes, one per rank, each rank holding only its stripe + S-row ref halo;
  the per-stripe MV records are gathered to rank 0 with one RCCL gather inside
  the timed step (strong scaling).
For N > 1 launch with torch.distributed.run (one process per GPU, RCCL).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
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
VALU_PEAK_ABSDIFF = 157.3e12  # 256 CU x 64 lanes x 2.4 GHz x 4 |a-b| per op (measured: profiles/)
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
    ap.add_argument("--mode", choices=["frames", "stripe"], default="frames")
    ap.add_argument("--config", choices=list(CONFIGS), default="1080p")
    ap.add_argument("--cost", choices=["sad", "ssd", "ssim"], default="sad")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-ssd", action="store_true",
                    help="skip the SSD (matrix-core) line beside a SAD run")
    ap.add_argument("--no-stream", action="store_true",
                    help="skip the host frame-pair streaming leg (PCIe-inclusive, not `value`)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL (production); gloo only to rehearse N ranks on one GPU")
    return ap.parse_args()


def _block_candidates(w, h, blk, span, bx, by):
    """Exact candidates of one block under the reference's clamping (main.c:73-76)."""
    tlx, tly = bx * blk, by * blk
    bw, bh = min(blk, w - tlx), min(blk, h - tly)
    nx = min(span, w - bw - tlx) - max(-span, -tlx) + 1
    ny = min(span, h - bh - tly) - max(-span, -tly) + 1
    return nx * ny


def cpu_baselines(ref, cur, blk, span, cost, threads, cands):
    """Rank 0, N=1 only: the oracle restatement (port) timed on the host cores
    on the same frame pair, and the reference's own binary (oracle/_ref/mes,
    MSE cost, its hard-coded 100-thread pool) when it was built."""
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
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        O.full_search(ref, cur, blk, span, cost, threads=threads, begin=begin, end=end)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    out = {"value": cands / med, "unit": "candidates/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model, "host_cpus": os.cpu_count(),
           "sample": f"{what} {w}x{h} B{blk} +-{span} {cost.upper()} frame, "
                     f"oracle/me_oracle.c -O2, {threads} pthreads, median of 5 ({med*1e3:.1f} ms)"}
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
    return out


def host_stream(eng, w, h, blk, span, cost, seed, sx, sy, kern_ms, cands_frame):
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
    for name, frames in (("pinned", list(pinned)), ("pageable", list(pageable))):
        eng.search_pairs(frames, pairs, blk, span, cost)  # allocates the device slots
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.search_pairs(frames, pairs, blk, span, cost)
        dt = (time.perf_counter() - t0) / reps
        out[name] = {"pairs_per_s": npairs / dt, "candidates_per_s": cands_frame * npairs / dt,
                     "ms_per_pair": dt / npairs * 1e3}
    out["kernel_only_pairs_per_s"] = 1e3 / kern_ms
    del pinned
    return out


def ssd_beside(eng, ref_t, cur_t, blk, span, nb, cands_frame, dev, steps):
    """The reference's own cost (MSE = SSD / 256) on the same resident frame pair:
    B = 16 SSD runs on the matrix cores (i8 MFMA).  Reported beside `value`."""
    import torch
    mv = torch.empty((nb, 2), dtype=torch.int16, device=dev)
    co = torch.empty(nb, dtype=torch.int32, device=dev)
    for _ in range(3):
        eng.full_search_device(ref_t, cur_t, blk, span, "ssd", mv, co)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(steps):
        eng.full_search_device(ref_t, cur_t, blk, span, "ssd", mv, co)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    tops = 2.0 * blk * blk * cands_frame / (ms / 1e3) / 1e12
    return {"value": cands_frame / (ms / 1e3), "unit": "candidates/s", "kernel_ms": ms,
            "steps": steps, "cost": "ssd (reference MSE argmin, bit-exact)",
            "roofline": {"bound": "mfma", "achieved": tops, "peak": I8_PEAK_TOPS,
                         "unit": "TFLOP/s", "frac": tops / I8_PEAK_TOPS}}


def load_traffic(tag):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this
    workload (tools/profile.sh), or None."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(tag, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    ndev = torch.cuda.device_count()
    gpu = local % ndev  # ranks > devices only in a gloo rehearsal on one GPU
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    gloo = args.dist_backend == "gloo"
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    import motionestimation_amd as me
    from motionestimation_amd import shard, synth

    cfg, blk, span = CONFIGS[args.config]
    w, h, seed, sx, sy = synth.CONFIGS[cfg]
    cands_frame = me.candidate_count(w, h, blk, span)
    nb = me.num_blocks(w, h, blk)
    eng = me.Engine(devices=[gpu])

    if args.mode == "frames":
        # rank r: its own frame pair of the sequence (same size; seed varies)
        ref, cur = synth.frame_pair(w, h, seed + rank, sx, sy)
        ref_t = torch.from_numpy(ref).to(dev)
        cur_t = torch.from_numpy(cur).to(dev)
        mv_t = torch.empty((nb, 2), dtype=torch.int16, device=dev)
        cost_t = torch.empty(nb, dtype=torch.int32, device=dev)

        def step():
            eng.full_search_device(ref_t, cur_t, blk, span, args.cost, mv_t, cost_t)
        units_per_step = cands_frame * world
    else:
        ref, cur = synth.frame_pair(w, h, seed, sx, sy)
        stripes = shard.plan(w, h, blk, span, world)
        st = stripes[rank]
        ref_t = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).to(dev)
        cur_t = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).to(dev)
        rec = torch.zeros((2, st.max_blocks), dtype=torch.int32, device=dev)
        mv_view = rec[0].view(torch.int16).view(st.max_blocks, 2)
        cost_view = rec[1]
        cdev = torch.device("cpu") if gloo else dev
        bufs = [torch.empty_like(rec, device=cdev) for _ in range(world)] if rank == 0 else None

        def step():
            if st.nblocks:
                eng.search_stripe_device(ref_t, st.ref_y0, cur_t, st.cur_y0, w, h, blk, span,
                                         args.cost, st.row_begin, st.row_end, mv_view, cost_view)
            if world > 1:  # the one exchange: per-stripe MV records -> rank 0 (RCCL)
                dist.gather(rec.cpu() if gloo else rec, bufs, dst=0)
        units_per_step = cands_frame

    # warmup (untimed)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # Kernel duration: one HIP event pair on the stream the search is launched
    # on (torch's current stream) around the whole timed region, / K.  Per-step
    # event pairs would insert a marker between every two launches and stretch
    # the measured step; the region average is the back-to-back launch time.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64,
                         device="cpu" if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    parity = None
    if args.mode == "stripe" and rank == 0 and world > 1:
        # the gathered field equals a single-GPU full-frame search (not timed)
        gmv, gcost = shard.assemble(bufs, stripes)
        fmv = torch.empty((nb, 2), dtype=torch.int16, device=dev)
        fco = torch.empty(nb, dtype=torch.int32, device=dev)
        eng.full_search_device(torch.from_numpy(ref).to(dev), torch.from_numpy(cur).to(dev), blk,
                               span, args.cost, fmv, fco)
        torch.cuda.synchronize()
        parity = bool(np.array_equal(gmv, fmv.cpu().numpy()) and
                      np.array_equal(gcost, fco.cpu().numpy().view(np.uint32)))

    value = units_per_step * args.steps / elapsed
    # Roofline of the dominant kernel: algorithmic HBM bytes per
    # launch = 2*W*H (u8 ref + cur, read once) + 8*nblocks (mv + cost written)
    # for the planes that launch covers.
    if args.mode == "frames":
        alg_bytes = 2 * w * h + 8 * nb
        absdiffs = cands_frame * blk * blk
    else:
        alg_bytes = (st.ref_y1 - st.ref_y0 + st.cur_y1 - st.cur_y0) * w + 8 * st.nblocks
        absdiffs = cands_frame * blk * blk / world
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9
    tag = f"{args.config}_b{blk}_s{span}_{args.cost}"
    traffic = load_traffic(tag)
    line = {
        "metric": METRIC if args.config == "1080p" and args.cost == "sad" else
        f"{blk}x{blk} {args.cost.upper()} candidates/sec at {args.config} +-{span}",
        "value": value,
        "unit": "candidates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if args.mode == "frames" else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic: motionestimation_amd.synth '{cfg}' (splitmix64 seed {seed}"
                f"{'+rank' if args.mode == 'frames' else ''}, 5x5 box, cur = ref shifted "
                f"({sx:+d},{sy:+d}) + uniform [-2,2])",
        "config": {"workload": f"{w}x{h} Y, {blk}x{blk} blocks, full search +-{span}, "
                               f"{args.cost.upper()}, {'one frame pair per rank per step' if args.mode == 'frames' else 'one frame per step in row stripes + RCCL gather'}",
                   "width": w, "height": h, "block": blk, "range": span, "cost": args.cost,
                   "candidates_per_frame": cands_frame, "blocks_per_frame": nb,
                   "parallelism": f"{args.mode}{world}"},
        "kernel_ms": kern_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": alg_bytes,
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
        ops = 2.0 * blk * blk * (cands_frame if args.mode == "frames" else cands_frame / world)
        tops = ops / (kern_ms / 1e3) / 1e12
        hbm = line["roofline"]
        hbm.pop("valu", None)
        line["roofline"] = {"bound": "mfma", "achieved": tops, "peak": I8_PEAK_TOPS,
                            "unit": "TFLOP/s", "frac": tops / I8_PEAK_TOPS, "traffic": traffic,
                            "note": "useful int8 ops (2*B*B per candidate) over the whole search "
                                    "(S2 prepass + MFMA kernel); dense i8 peak",
                            "hbm": {k: hbm[k] for k in ("achieved", "peak", "unit", "frac",
                                                        "algorithmic_bytes_per_launch")}}
    if (rank == 0 and world == 1 and args.mode == "frames" and args.cost == "sad"
            and blk == 16 and not args.no_ssd):
        line["ssd_mfma"] = ssd_beside(eng, ref_t, cur_t, blk, span, nb, cands_frame, dev,
                                      min(args.steps, 20))
    if parity is not None:
        line["stripe_gather_parity"] = parity
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baselines(ref, cur, blk, span, args.cost, args.cpu_threads,
                                             cands_frame)
    if rank == 0 and world == 1 and args.mode == "frames" and not args.no_stream:
        line["host_stream"] = host_stream(eng, w, h, blk, span, args.cost, seed, sx, sy,
                                          kern_ms, cands_frame)
    if rank == 0:
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
