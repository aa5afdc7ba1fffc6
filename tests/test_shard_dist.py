"""Row-stripe sharding with a real torch.distributed gather (gloo, world size 2
and 3, CPU).  Each rank sees ONLY its stripe's planes (cur stripe + S-row ref
halo): rows outside them are replaced by noise, so a wrong halo changes the
result.  The per-stripe compute here is the oracle (the GPU runs the same
stripe through me_full_search_stripe_device in test_gpu_parity)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_lib as O
from motionestimation_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stripe_search(ref, cur, st, blk, span, cost):
    rng = np.random.default_rng(99 + st.rank)
    h = ref.shape[0]
    ref_v = rng.integers(0, 256, ref.shape, dtype=np.uint8)
    cur_v = rng.integers(0, 256, cur.shape, dtype=np.uint8)
    ref_v[st.ref_y0:st.ref_y1] = ref[st.ref_y0:st.ref_y1]
    cur_v[st.cur_y0:st.cur_y1] = cur[st.cur_y0:st.cur_y1]
    b0 = st.row_begin * st.nbx
    mv, c, _ = O.full_search(ref_v, cur_v, blk, span, cost, threads=2, begin=b0,
                             end=b0 + st.nblocks)
    assert h == cur.shape[0]
    return mv, c


def _worker(rank, world, port, blk, span, cost, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        man = O.manifest()
        cur, ref = O.load_frame("ForemanYF2", man), O.load_frame("ForemanYF1", man)
        stripes = shard.plan(352, 288, blk, span, world)
        st = stripes[rank]
        mv, c = _stripe_search(ref, cur, st, blk, span, cost)
        rec = torch.from_numpy(shard.pack_records(mv, c, st.max_blocks))
        out = shard.gather_to_root(rec, stripes)
        if rank == 0:
            q.put((out[0].copy(), out[1].copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,blk,span,cost", [(2, 16, 16, "ssd"), (3, 8, 12, "sad")])
def test_stripe_gather_matches_full_frame(world, blk, span, cost):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, blk, span, cost, q))
             for r in range(world)]
    for p in procs:
        p.start()
    mv, c = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    man = O.manifest()
    cur, ref = O.load_frame("ForemanYF2", man), O.load_frame("ForemanYF1", man)
    emv, ec, _ = O.full_search(ref, cur, blk, span, cost)
    np.testing.assert_array_equal(mv, emv)
    np.testing.assert_array_equal(c, ec)


def test_stripe_extents_cover_halo():
    for st in shard.plan(1920, 1080, 16, 32, 8):
        assert st.ref_y0 == max(0, st.row_begin * 16 - 32)
        assert st.ref_y1 == min(1080, st.row_end * 16 + 32)
        assert st.cur_y1 - st.cur_y0 <= (st.row_end - st.row_begin) * 16
    sts = shard.plan(1920, 1080, 16, 32, 8)
    assert sum(s.nblocks for s in sts) == 120 * 68
