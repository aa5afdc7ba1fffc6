"""Host-side engine over libme_hip.so.

``Engine.full_search`` is the frame-level drop-in for the reference's dispatch
region (src/cpu/main.c:144-158): one call searches every block of the frame on
the GPU and returns the MV field plus per-block cost.  ``full_search_device``
works on HBM-resident torch tensors and enqueues on a stream (what bench.py
times); ``search_stripe_device`` is the per-rank unit of the row-stripe shard.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import ME_COST_SAD, ME_COST_SSD, ME_COST_SSIM, MEError, check

_COST = {"ssd": ME_COST_SSD, "mse": ME_COST_SSD, "sad": ME_COST_SAD, "ssim": ME_COST_SSIM,
         ME_COST_SSD: ME_COST_SSD, ME_COST_SAD: ME_COST_SAD, ME_COST_SSIM: ME_COST_SSIM}


def cost_code(cost) -> int:
    try:
        return _COST[cost]
    except KeyError:
        raise MEError(_lib.ME_EINVAL, f"unknown cost {cost!r}") from None


def num_blocks(width: int, height: int, blk: int) -> int:
    return int(_lib.lib().me_num_blocks(width, height, blk))


def candidate_count(width: int, height: int, blk: int, span: int) -> int:
    return int(_lib.lib().me_candidate_count(width, height, blk, span))


def plan_stripes(width: int, height: int, blk: int, span: int, shards: int) -> list:
    """Block-row boundaries [b0=0, ..., b_n=nby] balancing the kernels' cost
    model (me_plan_stripes, include/me.h): a block row costs
    nbx * (3 (2S+1) + ny), so a clipped edge row is discounted by a quarter of
    its candidate deficit, not all of it."""
    out = (ctypes.c_int * (shards + 1))()
    check(_lib.lib().me_plan_stripes(width, height, blk, span, shards, out))
    return list(out)


_PATH_CODES = {"auto": 0, "valu": 1, "tiles": 2, "lean": 3, "prepass": 4}


def set_kernel_path(path: str) -> None:
    """'auto': 16x16 and 8x8 SSD on the matrix cores (i8 MFMA; 16x16 with
    S <= 64 on the band-walk kernel when a launch's strips fill the CUs, else
    the prepass + block-major pair), the rest on the VALU kernels; 'valu':
    VALU kernels only; 'tiles': as 'auto' with 16x16 SSD on the 4x4-block-tile
    MFMA kernel; 'lean': 16x16 SSD (S <= 64) on the band-walk kernel for every
    launch (no prepass planes, no scratch); 'prepass': 16x16 SSD on the S2
    prepass + block-major pair.  Process-wide; results are identical."""
    if path not in _PATH_CODES:
        raise MEError(_lib.ME_EINVAL, f"unknown kernel path {path!r}")
    _lib.lib().me_set_kernel_path(_PATH_CODES[path])


SEARCH_PATHS = {0: "none", 1: "valu", 2: "mfma_prepass", 3: "mfma_bandwalk", 4: "mfma_lean",
                5: "mfma_tiles", 6: "mfma_8x8", 7: "ssim"}


def last_search_path() -> str:
    """The kernel family of the most recent search launched in this process
    (me_last_search_path): 'valu', 'mfma_prepass', 'mfma_bandwalk', ..."""
    return SEARCH_PATHS.get(_lib.lib().me_last_search_path(), "unknown")


def version() -> str:
    return _lib.lib().me_version().decode()


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class Engine:
    """One context: device buffers, a HIP stream per device, RCCL comms when
    created over several distinct devices.  Use from one thread at a time."""

    def __init__(self, devices=None):
        L = _lib.lib()
        h = ctypes.c_void_p()
        if devices:
            ids = (ctypes.c_int * len(devices))(*devices)
            st = L.me_create(ctypes.byref(h), ids, len(devices))
        else:
            st = L.me_create(ctypes.byref(h), None, 0)
        check(st)
        self._h = h
        self.devices = list(devices) if devices else None
        self.comm_ranks = 0  # me_comm_init: size of this context's RCCL group

    def set_kernel_path(self, path) -> None:
        """This context's kernel path (me_ctx_set_kernel_path): one of
        set_kernel_path()'s names, or None to follow the process-wide path."""
        if path is not None and path not in _PATH_CODES:
            raise MEError(_lib.ME_EINVAL, f"unknown kernel path {path!r}")
        code = _lib.ME_PATH_PROCESS if path is None else _PATH_CODES[path]
        check(_lib.lib().me_ctx_set_kernel_path(self._h, code), self._h)

    def last_search_path(self, device_index: int = 0) -> str:
        """The kernel family of this context's latest search on its device
        `device_index` (me_ctx_last_search_path)."""
        return SEARCH_PATHS.get(_lib.lib().me_ctx_last_search_path(self._h, device_index), "unknown")

    def close(self) -> None:
        if getattr(self, "_h", None):
            for g in getattr(self, "_graphs", ()):
                g.close()
            _lib.lib().me_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------- host API
    def full_search(self, ref, cur, blk: int, span: int, cost="ssd", stride=None):
        """Search (H, W) uint8 planes.  Returns (mv int16 [nblocks, 2] as
        (mvx, mvy), cost uint32 [nblocks]) in the reference's raster order."""
        ref = np.ascontiguousarray(ref, dtype=np.uint8)
        cur = np.ascontiguousarray(cur, dtype=np.uint8)
        if ref.ndim != 2 or ref.shape != cur.shape:
            raise MEError(_lib.ME_EINVAL, f"plane shapes {ref.shape} vs {cur.shape}")
        h, w = ref.shape
        n = num_blocks(w, h, blk) if blk > 0 else 0
        mv = np.zeros((max(n, 1), 2), np.int16)
        cst = np.zeros(max(n, 1), np.uint32)
        check(_lib.lib().me_full_search(self._h, _ptr(ref), _ptr(cur), w, h, stride or w, blk,
                                        span, cost_code(cost), _ptr(mv), _ptr(cst)), self._h)
        return mv[:n], cst[:n]

    def compensate_planes(self, ref, cur, blk: int, mv):
        """5-plane output [ref, cur, mc, |ref-cur|, |mc-cur|] (5H, W) and PSNR."""
        ref = np.ascontiguousarray(ref, np.uint8)
        cur = np.ascontiguousarray(cur, np.uint8)
        mv = np.ascontiguousarray(mv, np.int16)
        h, w = ref.shape
        out = np.zeros((5 * h, w), np.uint8)
        psnr = ctypes.c_double()
        check(_lib.lib().me_compensate_planes(self._h, _ptr(ref), _ptr(cur), w, h, blk,
                                              _ptr(mv), _ptr(out), ctypes.byref(psnr)), self._h)
        return out, psnr.value

    def motion_compensate(self, ref, blk: int, mv):
        ref = np.ascontiguousarray(ref, np.uint8)
        mv = np.ascontiguousarray(mv, np.int16)
        h, w = ref.shape
        mc = np.zeros_like(ref)
        check(_lib.lib().me_motion_compensate(self._h, _ptr(ref), w, h, blk, _ptr(mv),
                                              _ptr(mc)), self._h)
        return mc

    def search_pairs(self, frames, pairs, blk: int, span: int, cost="ssd"):
        """Search many (ref, cur) frame pairs in one pipelined call.

        frames: sequence of (H, W) uint8 planes (or one (N, H, W) array); pairs:
        [(ref_index, cur_index), ...].  Returns (mv int16 [npairs, nblocks, 2],
        cost uint32 [npairs, nblocks]).  Frames allocated with
        :func:`pinned_frames` are DMAed without staging."""
        # contiguous u8 frames pass through uncopied (pinned ones stay pinned)
        planes = [np.ascontiguousarray(f, dtype=np.uint8) for f in frames]
        if not planes:
            raise MEError(_lib.ME_EINVAL, "no frames")
        h, w = planes[0].shape
        for f in planes:
            if f.shape != (h, w):
                raise MEError(_lib.ME_EINVAL, f"frame shape {f.shape} != {(h, w)}")
        pr = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1, 2))
        npairs = pr.shape[0]
        n = num_blocks(w, h, blk) if blk > 0 else 0
        mv = np.zeros((max(npairs, 1), max(n, 1), 2), np.int16)
        cst = np.zeros((max(npairs, 1), max(n, 1)), np.uint32)
        ptrs = (ctypes.c_void_p * len(planes))(*[f.ctypes.data for f in planes])
        check(_lib.lib().me_search_pairs(self._h, ptrs, len(planes), w, h, w, blk, span,
                                         cost_code(cost), _ptr(pr), npairs, _ptr(mv),
                                         _ptr(cst)), self._h)
        return mv[:npairs, :n], cst[:npairs, :n]

    # ----------------------------------------------------------- device API
    def full_search_device(self, ref_t, cur_t, blk: int, span: int, cost, mv_t, cost_t=None,
                           stream=None, width=None, height=None, stride=None):
        """Enqueue a search on HBM-resident uint8 torch tensors (H, W); mv_t is an
        int16 tensor [nblocks, 2], cost_t uint32/int32 [nblocks] or None."""
        h, w = (height, width) if height else tuple(ref_t.shape[-2:])
        st = stream if stream is not None else _current_stream()
        check(_lib.lib().me_full_search_device(
            self._h, ref_t.data_ptr(), cur_t.data_ptr(), w, h, stride or w, blk, span,
            cost_code(cost), mv_t.data_ptr(), cost_t.data_ptr() if cost_t is not None else None,
            st), self._h)

    def search_stripe_device(self, ref_t, ref_row0: int, cur_t, cur_row0: int, width: int,
                             height: int, blk: int, span: int, cost, row_begin: int,
                             row_end: int, mv_t, cost_t=None, stream=None, stride=None):
        """One row stripe (block rows [row_begin, row_end)) on resident planes that
        start at frame rows ref_row0 / cur_row0."""
        st = stream if stream is not None else _current_stream()
        check(_lib.lib().me_full_search_stripe_device(
            self._h, ref_t.data_ptr(), ref_row0, cur_t.data_ptr(), cur_row0, width, height,
            stride or width, blk, span, cost_code(cost), row_begin, row_end, mv_t.data_ptr(),
            cost_t.data_ptr() if cost_t is not None else None, st), self._h)


    def search_stripes_device(self, width: int, height: int, blk: int, span: int, cost, jobs,
                              stream=None, stride=None):
        """Several stripes in one call (me_search_stripes_device).  jobs: list of
        (ref_t, ref_row0, cur_t, cur_row0, row_begin, row_end, mv_t, cost_t) --
        the arguments of one search_stripe_device each (tensors (rows, pitch))."""
        self.prepared_stripes_search(width, height, blk, span, cost, jobs, stream, stride)()

    def prepared_stripes_search(self, width, height, blk, span, cost, jobs, stream=None,
                                stride=None):
        """Zero-argument callable enqueueing search_stripes_device(...) with these buffers."""
        arr = (StripeJob * len(jobs))()
        for a, (rt, r0, ct, c0, b0, b1, mv, co) in zip(arr, jobs):
            a.d_ref, a.ref_row0, a.d_cur, a.cur_row0 = rt.data_ptr(), r0, ct.data_ptr(), c0
            a.block_row_begin, a.block_row_end = b0, b1
            a.d_mv_xy, a.d_block_cost = mv.data_ptr(), co.data_ptr() if co is not None else None
        pitch = stride or jobs[0][0].stride(0) * jobs[0][0].element_size()
        fn, h = _lib.lib().me_search_stripes_device, self._h
        args = (h, width, height, pitch, blk, span, cost_code(cost), arr, len(jobs),
                stream if stream is not None else _current_stream())

        def run():
            s = fn(*args)
            if s:
                check(s, h)
        run.jobs = arr  # keep the descriptor array alive with the callable
        return run

    def search_batch_device(self, ref_t, ref_row0: int, cur_t, cur_row0: int, width: int,
                            height: int, blk: int, span: int, cost, row_begin: int, row_end: int,
                            mv_t, cost_t=None, stream=None, stride=None):
        """A batch of stripes in one launch (me_full_search_batch_device):
        ref_t / cur_t are uint8 tensors [F, rows, pitch] (frame f = ref_t[f]),
        mv_t int16 [F * nblk, 2] and cost_t [F * nblk], frame-major."""
        st = stream if stream is not None else _current_stream()
        check(_lib.lib().me_full_search_batch_device(*self._batch_args(
            ref_t, ref_row0, cur_t, cur_row0, width, height, blk, span, cost, row_begin, row_end,
            mv_t, cost_t, st, stride)), self._h)

    def _batch_args(self, ref_t, ref_row0, cur_t, cur_row0, width, height, blk, span, cost,
                    row_begin, row_end, mv_t, cost_t, stream, stride):
        if ref_t.dim() != 3 or cur_t.dim() != 3 or ref_t.shape[0] != cur_t.shape[0]:
            raise MEError(_lib.ME_EINVAL, f"batch shapes {tuple(ref_t.shape)} / {tuple(cur_t.shape)}")
        es = ref_t.element_size()
        return (self._h, ref_t.data_ptr(), ref_t.stride(0) * es, ref_row0, cur_t.data_ptr(),
                cur_t.stride(0) * es, cur_row0, width, height, stride or ref_t.stride(1) * es,
                blk, span, cost_code(cost), row_begin, row_end, ref_t.shape[0],
                mv_t.data_ptr(), cost_t.data_ptr() if cost_t is not None else None, stream)

    def prepared_batch_search(self, ref_t, ref_row0, cur_t, cur_row0, width, height, blk, span,
                              cost, row_begin, row_end, mv_t, cost_t, stream=None, stride=None):
        """Zero-argument callable enqueueing search_batch_device(...) with these buffers."""
        fn, h = _lib.lib().me_full_search_batch_device, self._h
        args = self._batch_args(ref_t, ref_row0, cur_t, cur_row0, width, height, blk, span, cost,
                                row_begin, row_end, mv_t, cost_t,
                                stream if stream is not None else _current_stream(), stride)

        def run():
            s = fn(*args)
            if s:
                check(s, h)
        return run

    # ---- multi-process stripes: the one exchange step in native code ----
    @staticmethod
    def comm_unique_id() -> bytes:
        """RCCL unique id (rank 0), to be sent to every rank out of band."""
        buf = ctypes.create_string_buffer(_lib.ME_COMM_ID_BYTES)
        check(_lib.lib().me_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, uid: bytes, n_ranks: int, rank: int) -> None:
        """Join an n_ranks RCCL group on this context's first device (collective)."""
        if len(uid) != _lib.ME_COMM_ID_BYTES:
            raise ValueError(f"comm id of {len(uid)} bytes, expected {_lib.ME_COMM_ID_BYTES}")
        check(_lib.lib().me_comm_init(self._h, uid, n_ranks, rank), self._h)
        self.comm_ranks = n_ranks

    def gather_device(self, send_t, recv_t=None, stream=None) -> None:
        """Gather send_t (same byte count on every rank) into rank 0's recv_t
        (n_ranks x the bytes, rank order), enqueued on `stream` (default: torch's
        current stream)."""
        st = stream if stream is not None else _current_stream()
        check(_lib.lib().me_gather_device(
            self._h, send_t.data_ptr(), send_t.numel() * send_t.element_size(),
            recv_t.data_ptr() if recv_t is not None else None, st), self._h)


    def comm_check(self, timeout_ms: int = _lib.ME_COMM_TIMEOUT_MS, stream=None) -> None:
        """Bounded wait for the work on `stream` (default: torch's current
        stream) with RCCL failure detection (me_comm_check): raises MEError
        (ME_ECOMM) on an RCCL error or when timeout_ms passed; the communicator
        is then aborted."""
        st = stream if stream is not None else _current_stream()
        check(_lib.lib().me_comm_check(self._h, st, int(timeout_ms)), self._h)

    def device_check(self) -> None:
        """Raise MEError (ME_EDEVICE) if a search kernel reported a broken
        in-kernel invariant since the last check (call after synchronising)."""
        check(_lib.lib().me_device_check(self._h), self._h)

    # ---- captured steps: one graph launch per frame ----
    def capture(self, stream, enqueue) -> "Graph":
        """Record what enqueue() puts on `stream` (device entry points of this
        context, e.g. a stripe search and its gather) as one graph.  Run the
        searches once uncaptured first (they size the context's scratch)."""
        L = _lib.lib()
        check(L.me_capture_begin(self._h, stream), self._h)
        g = ctypes.c_void_p()
        try:
            enqueue()
        except BaseException:
            # end the capture (the stream must leave capture mode) and drop the
            # graph it made; the enqueue's exception is the one that propagates
            if L.me_capture_end(self._h, stream, ctypes.byref(g)) == _lib.ME_OK and g:
                L.me_graph_destroy(g)
            raise
        st = L.me_capture_end(self._h, stream, ctypes.byref(g))
        check(st, self._h)
        gr = Graph(self, g)
        if not hasattr(self, "_graphs"):
            self._graphs = []
        self._graphs.append(gr)  # destroyed before the context (include/me.h)
        return gr

    # ---- prepared calls: arguments marshalled once per buffer set ----
    # A sharded step on a small stripe is bound by host time (an 8-way 1080p
    # stripe searches in 15-18 us), so the per-frame calls skip the wrapper's
    # argument handling.  The caller keeps the tensors alive.
    def prepared_stripe_search(self, ref_t, ref_row0, cur_t, cur_row0, width, height, blk,
                               span, cost, row_begin, row_end, mv_t, cost_t, stream=None,
                               stride=None):
        """Zero-argument callable enqueueing search_stripe_device(...) with these
        fixed buffers on `stream` (default: torch's current stream now)."""
        fn, h = _lib.lib().me_full_search_stripe_device, self._h
        args = (h, ref_t.data_ptr(), ref_row0, cur_t.data_ptr(), cur_row0, width, height,
                stride or width, blk, span, cost_code(cost), row_begin, row_end,
                mv_t.data_ptr(), cost_t.data_ptr() if cost_t is not None else None,
                stream if stream is not None else _current_stream())

        def run():
            s = fn(*args)
            if s:
                check(s, h)
        return run

    def prepared_gather(self, send_t, recv_t=None, stream=None):
        """Zero-argument callable enqueueing gather_device(send_t, recv_t)."""
        fn, h = _lib.lib().me_gather_device, self._h
        args = (h, send_t.data_ptr(), send_t.numel() * send_t.element_size(),
                recv_t.data_ptr() if recv_t is not None else None,
                stream if stream is not None else _current_stream())

        def run():
            s = fn(*args)
            if s:
                check(s, h)
        return run


class StripeJob(ctypes.Structure):
    """include/me.h me_stripe_job."""
    _fields_ = [("d_ref", ctypes.c_void_p), ("ref_row0", ctypes.c_int),
                ("d_cur", ctypes.c_void_p), ("cur_row0", ctypes.c_int),
                ("block_row_begin", ctypes.c_int), ("block_row_end", ctypes.c_int),
                ("d_mv_xy", ctypes.c_void_p), ("d_block_cost", ctypes.c_void_p)]


class Graph:
    """A captured step (me_capture_begin/end); launch() replays it on a stream."""

    def __init__(self, eng: Engine, handle):
        self._eng, self._h = eng, handle
        self._launch = _lib.lib().me_graph_launch

    def launch(self, stream) -> None:
        s = self._launch(self._h, stream)
        if s:
            check(s, self._eng._h)

    def prepared(self, stream):
        """Zero-argument callable launching the graph on `stream`."""
        fn, h, ctx = self._launch, self._h, self._eng._h

        def run():
            s = fn(h, stream)
            if s:
                check(s, ctx)
        return run

    def set_kernel_path(self, path) -> None:
        """This context's kernel path (me_ctx_set_kernel_path): one of
        set_kernel_path()'s names, or None to follow the process-wide path."""
        if path is not None and path not in _PATH_CODES:
            raise MEError(_lib.ME_EINVAL, f"unknown kernel path {path!r}")
        code = _lib.ME_PATH_PROCESS if path is None else _PATH_CODES[path]
        check(_lib.lib().me_ctx_set_kernel_path(self._h, code), self._h)

    def last_search_path(self, device_index: int = 0) -> str:
        """The kernel family of this context's latest search on its device
        `device_index` (me_ctx_last_search_path)."""
        return SEARCH_PATHS.get(_lib.lib().me_ctx_last_search_path(self._h, device_index), "unknown")

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().me_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Pinned:
    """Owner of one me_host_alloc block (freed when the last view dies)."""

    def __init__(self, nbytes: int):
        self.ptr = _lib.lib().me_host_alloc(nbytes)
        if not self.ptr:
            raise MEError(_lib.ME_ENOMEM, f"me_host_alloc({nbytes})")

    def __del__(self):
        if getattr(self, "ptr", None):
            try:
                _lib.lib().me_host_free(self.ptr)
            except Exception:  # interpreter shutdown: module globals already torn down
                pass
            self.ptr = None


def pinned_frames(n: int, height: int, width: int) -> np.ndarray:
    """(n, height, width) uint8 array in pinned host memory (me_host_alloc):
    frames written here are uploaded by DMA without a staging copy."""
    owner = _Pinned(max(1, n * height * width))
    buf = (ctypes.c_uint8 * (n * height * width)).from_address(owner.ptr)
    buf._owner = owner  # keep the allocation alive with every view
    return np.frombuffer(buf, dtype=np.uint8).reshape(n, height, width)


def _current_stream():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
