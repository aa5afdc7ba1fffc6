import sys, json, torch, ctypes
sys.path.insert(0, '/root/repo')
import motionestimation_amd as me
from motionestimation_amd import shard, synth
for cfg, blk, span in (("1080p", 16, 32), ("4k", 16, 64)):
    w, h, seed, sx, sy = synth.CONFIGS[cfg]
    ref, cur = synth.frame_pair(w, h, seed, sx, sy)
    st = shard.plan(w, h, blk, span, 8)[3]
    rt = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).cuda()
    ct = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).cuda()
    engs = [me.Engine(devices=[0]), me.Engine(devices=[0])]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [(torch.empty((st.nblocks, 2), dtype=torch.int16, device="cuda"),
             torch.empty(st.nblocks, dtype=torch.int32, device="cuda")) for _ in range(2)]
    for nstreams in (1, 2):
        def run(i):
            k = i % nstreams
            mv, co = outs[k]
            engs[k].search_stripe_device(rt, st.ref_y0, ct, st.cur_y0, w, h, blk, span, "sad",
                                         st.row_begin, st.row_end, mv, co,
                                         stream=ctypes.c_void_p(streams[k].cuda_stream))
        for i in range(10): run(i)
        torch.cuda.synchronize()
        import time
        t0 = time.perf_counter()
        n = 200
        for i in range(n): run(i)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        print(json.dumps({"config": cfg, "stripe": [st.row_begin, st.row_end], "streams": nstreams, "us_per_stripe": dt * 1e6}))
