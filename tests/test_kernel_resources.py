"""Scratch and spill budget of every kernel in libme_hip.so (CPU suite).

The built gfx950 code objects' metadata (`.private_segment_fixed_size`,
`.vgpr_spill_count`, read by tests/kernel_resources.py) is compared with the
committed ceilings in tests/kernel_budget.json: a kernel not listed there must
use no scratch at all.  Round 5's 4K SAD kernel regression (5 VGPRs spilled,
24 bytes per lane, 32.7 MiB of spill writes per launch) went unnoticed because
nothing checked this; the SAD kernel is me_fast_kernel (souravBhat/
MotionEstimation src/cpu/main.c:39-64 restated on the VALU).
"""
import json
import os

import pytest

import kernel_resources as kr

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "motionestimation_amd", "lib", "libme_hip.so")


@pytest.mark.skipif(not kr.tools_present(), reason="llvm-objcopy / llvm-readelf not installed")
def test_kernel_scratch_within_budget():
    if not os.path.exists(LIB):
        pytest.skip("libme_hip.so not built")
    with open(os.path.join(REPO, "tests", "kernel_budget.json")) as f:
        budget = json.load(f)["kernels"]
    ks = kr.kernels(LIB)
    assert len(ks) >= 40, f"expected the product's kernels, found {len(ks)}"
    names = kr.demangle(sorted(ks))
    over = []
    for mangled, r in ks.items():
        b = budget.get(names[mangled], {"scratch_bytes": 0, "vgpr_spills": 0})
        if r["private_segment_fixed_size"] > b["scratch_bytes"] or r["vgpr_spill_count"] > b["vgpr_spills"]:
            over.append(f"{names[mangled]}: {r['private_segment_fixed_size']} B scratch, "
                        f"{r['vgpr_spill_count']} VGPR spills (budget {b['scratch_bytes']} B, {b['vgpr_spills']})")
    assert not over, "kernels over their scratch budget:\n" + "\n".join(over)


@pytest.mark.skipif(not kr.tools_present(), reason="llvm-objcopy / llvm-readelf not installed")
def test_headline_kernels_spill_free():
    """The kernels the bench line and its legs time spill nothing."""
    if not os.path.exists(LIB):
        pytest.skip("libme_hip.so not built")
    ks = kr.kernels(LIB)
    names = kr.demangle(sorted(ks))
    for frag in ("me_flow_kernel<16, 13, 144>", "me_mfma_bw_kernel<4, 2, 160, 12, 4, false>",
                 "me_mfma_bm16_kernel<288>", "me_fast_kernel<1, 8, 26, 336>", "me_ssim_kernel"):
        hits = [m for m in ks if frag in names[m]]
        assert hits, frag
        for m in hits:
            assert ks[m]["private_segment_fixed_size"] == 0 and ks[m]["vgpr_spill_count"] == 0, names[m]
