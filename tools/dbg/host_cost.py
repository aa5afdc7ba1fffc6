"""Host time per call of the search entry points (no sync inside the loop):
is a small stripe search host-bound?"""
import ctypes, json, sys, time
import torch
sys.path.insert(0, '/root/repo')
import motionestimation_amd as me
from motionestimation_amd import _lib, shard, synth
w, h, seed, sx, sy = synth.CONFIGS["1080p"]
ref, cur = synth.frame_pair(w, h, seed, sx, sy)
st = shard.plan(w, h, 16, 32, 8)[3]
rt = torch.from_numpy(ref[st.ref_y0:st.ref_y1].copy()).cuda()
ct = torch.from_numpy(cur[st.cur_y0:st.cur_y1].copy()).cuda()
eng = me.Engine(devices=[0])
mv = torch.empty((st.nblocks, 2), dtype=torch.int16, device="cuda")
co = torch.empty(st.nblocks, dtype=torch.int32, device="cuda")
L = _lib.lib()
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
args = (eng._h, rt.data_ptr(), st.ref_y0, ct.data_ptr(), st.cur_y0, w, h, w, 16, 32, 1,
        st.row_begin, st.row_end, mv.data_ptr(), co.data_ptr(), sp)
def py_call():
    eng.search_stripe_device(rt, st.ref_y0, ct, st.cur_y0, w, h, 16, 32, "sad", st.row_begin, st.row_end, mv, co)
def raw_call():
    L.me_full_search_stripe_device(*args)
for name, fn in (("python wrapper", py_call), ("raw ctypes", raw_call)):
    for _ in range(20): fn()
    torch.cuda.synchronize()
    n = 300
    t0 = time.perf_counter()
    for _ in range(n): fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"call": name, "host_us_per_call": (t1 - t0) / n * 1e6, "wall_us_per_call": (t2 - t0) / n * 1e6}))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(300): raw_call()
e1.record(); torch.cuda.synchronize()
print(json.dumps({"call": "raw ctypes, event timing", "gpu_us_per_call": e0.elapsed_time(e1) / 300 * 1e3}))
