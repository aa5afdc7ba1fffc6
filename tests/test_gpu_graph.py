"""GPU: captured steps (me_capture_begin/end, me_graph_launch) and the
invariant check (me_device_check).

A rank's per-frame step -- its stripe search and the one RCCL gather -- is
captured once and replayed with one graph launch (bench.py's stripe mode).  The
replayed fields must equal direct searches and the oracle bit for bit; a
captured search that would grow the context's scratch, and a graph whose
scratch was regrown after capture, are refused with ME_EINVAL."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
import motionestimation_amd as me
from motionestimation_amd import shard, synth

pytestmark = pytest.mark.gpu


def _stream():
    import torch
    s = torch.cuda.Stream()
    return s, ctypes.c_void_p(s.cuda_stream)


@pytest.mark.parametrize("cost,blk,span,ways,rank", [
    ("sad", 16, 32, 8, 1),   # the 8-way 1080p stripe of bench.py (small-stripe item kernel)
    ("sad", 16, 32, 1, 0),   # whole frame: the flow kernel
    ("ssd", 16, 32, 4, 3),   # matrix cores: prepass + block-major kernel, bottom edge
    ("sad", 8, 24, 3, 2),    # 8x8 qsad
])
def test_captured_stripe_search_equals_oracle(cost, blk, span, ways, rank):
    import torch
    ref, cur = synth.frame_pair(1920, 1080, 11, 3, -2)
    st = shard.plan(1920, 1080, blk, span, ways)[rank]
    s, sh = _stream()
    with me.Engine(devices=[0]) as eng, torch.cuda.stream(s):
        rt = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).cuda()
        ct = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).cuda()
        mv = torch.full((st.max_blocks, 2), -7, dtype=torch.int16, device="cuda")
        co = torch.zeros(st.max_blocks, dtype=torch.int32, device="cuda")
        run = eng.prepared_stripe_search(rt, st.ref_y0, ct, st.cur_y0, 1920, 1080, blk, span, cost,
                                         st.row_begin, st.row_end, mv, co, stream=sh)
        run()  # uncaptured first: sizes the scratch
        torch.cuda.synchronize()
        g = eng.capture(sh, run)
        mv.fill_(-7)
        co.zero_()
        for _ in range(3):  # replays reuse the self-resetting counters
            g.launch(sh)
        torch.cuda.synchronize()
        eng.device_check()
        omv, oco, _ = O.full_search(ref, cur, blk, span, cost, threads=16,
                                    begin=st.row_begin * st.nbx, end=st.row_end * st.nbx)
        np.testing.assert_array_equal(mv[:st.nblocks].cpu().numpy(), omv)
        np.testing.assert_array_equal(co[:st.nblocks].cpu().numpy().view(np.uint32), oco)


def test_captured_search_and_gather_one_rank():
    """bench.py's graph: search + me_gather_device replayed alternately from two
    graphs (double-buffered records) in a one-rank library communicator."""
    import torch
    ref, cur = synth.frame_pair(1920, 1080, 12, -5, 4)
    st = shard.plan(1920, 1080, 16, 32, 8)[4]
    s, sh = _stream()
    with me.Engine(devices=[0]) as eng, torch.cuda.stream(s):
        eng.comm_init(eng.comm_unique_id(), 1, 0)
        rt = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).cuda()
        ct = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).cuda()
        recs = [torch.zeros((2, st.max_blocks), dtype=torch.int32, device="cuda") for _ in range(2)]
        flat = [torch.zeros((1, 2, st.max_blocks), dtype=torch.int32, device="cuda") for _ in range(2)]
        runs = []
        for k in range(2):
            mv = recs[k][0].view(torch.int16).view(st.max_blocks, 2)
            ps = eng.prepared_stripe_search(rt, st.ref_y0, ct, st.cur_y0, 1920, 1080, 16, 32,
                                            "sad", st.row_begin, st.row_end, mv, recs[k][1],
                                            stream=sh)
            pg = eng.prepared_gather(recs[k], flat[k], stream=sh)
            ps()
            pg()
            runs.append((ps, pg))
        torch.cuda.synchronize()
        graphs = [eng.capture(sh, lambda r=r: (r[0](), r[1]())) for r in runs]
        for f in flat:
            f.zero_()
        for i in range(10):
            graphs[i & 1].launch(sh)
        torch.cuda.synchronize()
        eng.device_check()
        omv, oco, _ = O.full_search(ref, cur, 16, 32, "sad", threads=16,
                                    begin=st.row_begin * st.nbx, end=st.row_end * st.nbx)
        for k in range(2):
            got = flat[k][0]
            assert torch.equal(got, recs[k])
            np.testing.assert_array_equal(
                got[0].cpu().numpy().view(np.int16).reshape(-1, 2)[:st.nblocks], omv)
            np.testing.assert_array_equal(got[1].cpu().numpy().view(np.uint32)[:st.nblocks], oco)


def test_capture_refuses_scratch_growth_and_stale_graphs():
    import torch
    ref, cur = synth.frame_pair(640, 480, 13, 2, 2)
    big_ref, big_cur = synth.frame_pair(1920, 1080, 13, 2, 2)
    s, sh = _stream()
    with me.Engine(devices=[0]) as eng, torch.cuda.stream(s):
        rt, ct = torch.from_numpy(ref).cuda(), torch.from_numpy(cur).cuda()
        n = me.num_blocks(640, 480, 16)
        mv = torch.empty((n, 2), dtype=torch.int16, device="cuda")
        co = torch.empty(n, dtype=torch.int32, device="cuda")

        def search():
            eng.full_search_device(rt, ct, 16, 16, "ssd", mv, co, stream=sh)
        # never run: the matrix-core search would allocate its prepass planes
        with pytest.raises(me.MEError) as ei:
            eng.capture(sh, search)
        assert ei.value.status == me._lib.ME_EINVAL
        search()
        torch.cuda.synchronize()
        g = eng.capture(sh, search)
        g.launch(sh)
        torch.cuda.synchronize()
        omv, oco, _ = O.full_search(ref, cur, 16, 16, "ssd", threads=16)
        np.testing.assert_array_equal(mv.cpu().numpy(), omv)
        # a bigger search regrows the scratch the graph points into
        eng.full_search(big_ref, big_cur, 16, 32, "ssd")
        with pytest.raises(me.MEError) as ei:
            g.launch(sh)
        assert ei.value.status == me._lib.ME_EINVAL


def test_device_check_clean_after_searches(engine):
    ref, cur = synth.frame_pair(352, 288, 3, 1, 1)
    for cost in ("sad", "ssd"):
        engine.full_search(ref, cur, 16, 16, cost)
    engine.device_check()
