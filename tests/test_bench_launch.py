"""bench.py's rank setup, on the CPU: `--gpus N` never degrades to a one-rank
line.  Without a launcher bench.py starts its own N ranks (launch_ranks); a
request for more RCCL ranks than visible GPUs, or a --gpus that disagrees with
the launcher's WORLD_SIZE, exits non-zero with nothing on stdout.  The spawn
itself is exercised on the GPU box (tests/test_gpu_multi.py)."""
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _gpus():
    import torch
    return torch.cuda.device_count()


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args, "--no-cpu"], capture_output=True,
                          text=True, timeout=120, env=env)


@pytest.mark.skipif("_gpus() >= 2", reason="the box has enough GPUs: the spawn would run")
def test_more_rccl_ranks_than_gpus_is_refused():
    r = _run(["--gpus", "2"])
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "visible GPUs" in r.stderr


def test_gpus_disagreeing_with_world_size_is_refused():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert "WORLD_SIZE" in r.stderr


def test_exact_absdiff_count():
    """roofline.valu bills w*h per block: the 1080p bottom row is 16x8."""
    sys.path.insert(0, REPO)
    import bench
    import motionestimation_amd as me
    assert bench.exact_absdiffs(1920, 1080, 16, 32) == 8_463_799_296
    # brute force on a small ragged frame against the per-block definition
    w, h, blk, span = 70, 45, 16, 9
    tot = 0
    for by in range((h + blk - 1) // blk):
        for bx in range((w + blk - 1) // blk):
            bw, bh = min(blk, w - bx * blk), min(blk, h - by * blk)
            tot += bench._block_candidates(w, h, blk, span, bx, by) * bw * bh
    assert bench.exact_absdiffs(w, h, blk, span) == tot
    assert me.candidate_count(w, h, blk, span) == sum(
        bench._block_candidates(w, h, blk, span, bx, by)
        for by in range(3) for bx in range(5))
    assert np.isclose(bench.exact_absdiffs(w, h, blk, span, 1, 2),
                      sum(bench._block_candidates(w, h, blk, span, bx, 1) * min(blk, w - bx * blk) * 16
                          for bx in range(5)))


def test_frames_per_launch_pricing():
    """bench.py prices the roofline per launch with the library's batching rules:
    SAD batches share one launch of up to MAX_JOBS frames, 8K 8x8 +-128
    included (me_kernels.hip launch_item_jobs); 8x8 SSD launches per frame."""
    sys.path.insert(0, REPO)
    import bench
    assert bench.sad_frames_per_launch(1920, 1080, 16, 32, 16) == 16
    assert bench.sad_frames_per_launch(3840, 2160, 16, 64, 16) == 16
    assert bench.sad_frames_per_launch(3840, 2160, 16, 64, 64) == bench.MAX_JOBS
    assert bench.sad_frames_per_launch(7680, 4320, 8, 128, 16) == 16
    assert bench.sad_frames_per_launch(7680, 68 * 8, 8, 128, 16) == 16
    assert bench.ssd_frames_per_launch(7680, 4320, 8, 128, 16) == 1


def test_committed_pmc_summary_feeds_the_roofline_figures():
    """bench.py reads its `traffic` and the 8x8 SSD line's `valu` figure from
    the committed profiles/pmc_summary.json (tools/profile.sh): the entries the
    default and 8K SSD lines need exist, and the VALU pass counts more VALU
    than MFMA wave-instructions (SQ_INSTS_VALU includes the MFMAs)."""
    sys.path.insert(0, REPO)
    import bench
    t, ts = bench.load_traffic("1080p_b16_s32_sad_f16")
    assert t and ts and t > 60e6
    v = bench.load_valu("8k_b8_s128_ssd_f16")
    assert v is not None and v["kernel"].startswith("me_mfma_ssd8_kernel")
    assert v["valu"] > v["mfma"] > 0
    assert bench.load_valu("no_such_workload") is None
