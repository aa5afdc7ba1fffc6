"""ctypes binding of libme_hip.so (include/me.h).  No fallback: if the HIP
library is missing or fails to load, every entry point raises."""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
LIB_PATH = os.path.join(PKG, "lib", "libme_hip.so")
# Diagnostic builds only (tuning tools, tools/stamps.py): another in-tree
# build of the same library.
if os.environ.get("ME_HIP_LIB"):
    LIB_PATH = os.path.join(PKG, "lib", os.path.basename(os.environ["ME_HIP_LIB"]))
CSRC = os.path.join(PKG, "csrc")

ME_OK, ME_EINVAL, ME_ENOMEM, ME_EDEVICE, ME_ECOMM, ME_EUNSUPPORTED, ME_EIO = range(7)
ME_COMM_ID_BYTES = 128  # include/me.h (sizeof ncclUniqueId)
ME_COMM_TIMEOUT_MS = 60000
ME_YUV_LUMA, ME_YUV_I420 = 0, 1
ME_COST_SSD, ME_COST_SAD, ME_COST_SSIM = 0, 1, 2
ME_PATH_AUTO, ME_PATH_VALU, ME_PATH_MFMA_TILES, ME_PATH_MFMA_LEAN, ME_PATH_MFMA_PREPASS = 0, 1, 2, 3, 4
ME_PATH_PROCESS = -1
ME_MAX_BLOCK, ME_MAX_RANGE = 64, 1024

# Every symbol include/me.h declares, with (restype, argtypes).
_u8p = ctypes.c_void_p
_SIGS = {
    "me_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int),
                                 ctypes.c_int]),
    "me_destroy": (None, [ctypes.c_void_p]),
    "me_status_str": (ctypes.c_char_p, [ctypes.c_int]),
    "me_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "me_version": (ctypes.c_char_p, []),
    "me_num_blocks": (ctypes.c_int, [ctypes.c_int] * 3),
    "me_set_kernel_path": (None, [ctypes.c_int]),
    "me_last_search_path": (ctypes.c_int, []),
    "me_ctx_set_kernel_path": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "me_ctx_last_search_path": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "me_candidate_count": (ctypes.c_uint64, [ctypes.c_int] * 4),
    "me_full_search": (ctypes.c_int, [ctypes.c_void_p, _u8p, _u8p] + [ctypes.c_int] * 6 +
                       [ctypes.c_void_p, ctypes.c_void_p]),
    "me_full_search_device": (ctypes.c_int, [ctypes.c_void_p, _u8p, _u8p] + [ctypes.c_int] * 6 +
                              [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "me_full_search_stripe_device": (ctypes.c_int, [ctypes.c_void_p, _u8p, ctypes.c_int, _u8p,
                                                    ctypes.c_int] + [ctypes.c_int] * 8 +
                                     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "me_full_search_batch_device": (ctypes.c_int, [ctypes.c_void_p, _u8p, ctypes.c_size_t,
                                                   ctypes.c_int, _u8p, ctypes.c_size_t] +
                                    [ctypes.c_int] * 10 +
                                    [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "me_search_stripes_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_int] * 6 +
                                 [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),  # jobs: me_stripe_job*
    "me_plan_stripes": (ctypes.c_int, [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_int)]),
    "me_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "me_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "me_gather_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "me_comm_check": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "me_device_check": (ctypes.c_int, [ctypes.c_void_p]),
    "me_capture_begin": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "me_capture_end": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_void_p)]),
    "me_graph_launch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "me_graph_destroy": (None, [ctypes.c_void_p]),
    "me_find_best_blocks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p] +
                            [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_int]),
    "me_motion_compensate": (ctypes.c_int, [ctypes.c_void_p, _u8p] + [ctypes.c_int] * 3 +
                             [ctypes.c_void_p, ctypes.c_void_p]),
    "me_compensate_planes": (ctypes.c_int, [ctypes.c_void_p, _u8p, _u8p] + [ctypes.c_int] * 3 +
                             [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "me_host_alloc": (ctypes.c_void_p, [ctypes.c_size_t]),
    "me_host_free": (None, [ctypes.c_void_p]),
    "me_search_pairs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 7 +
                        [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "me_yuv_frame_count": (ctypes.c_int64, [ctypes.c_char_p] + [ctypes.c_int] * 3),
    "me_yuv_read_luma": (ctypes.c_int, [ctypes.c_char_p] + [ctypes.c_int] * 4 +
                         [ctypes.c_void_p, ctypes.c_int]),
    "me_yuv_write": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_int]),
    "me_mv_write": (ctypes.c_int, [ctypes.c_char_p] + [ctypes.c_int] * 5 +
                    [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "me_mv_read_header": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_void_p]),
    "me_mv_read": (ctypes.c_int, [ctypes.c_char_p] + [ctypes.c_void_p] * 4),
}


class MEError(RuntimeError):
    def __init__(self, status: int, detail: str = ""):
        self.status = status
        name = _names.get(status, f"status {status}")
        super().__init__(f"{name}: {detail}" if detail else name)


_names = {ME_EINVAL: "ME_EINVAL", ME_ENOMEM: "ME_ENOMEM", ME_EDEVICE: "ME_EDEVICE",
          ME_ECOMM: "ME_ECOMM", ME_EUNSUPPORTED: "ME_EUNSUPPORTED", ME_EIO: "ME_EIO"}

_lib = None


def build(force: bool = False) -> str:
    """Compile libme_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    cmd = ["make", "-s", "-C", CSRC]
    if force:
        cmd.append("-B")
    subprocess.run(cmd, check=True)
    return LIB_PATH


def lib():
    """The loaded library; raises if it is absent (the product has no CPU path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with "
                               "`python -c 'import __graft_entry__; __graft_entry__.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("ME_HIP_LIB") and not hasattr(L, name):
                continue  # an older diagnostic build (A/B runs) may lack newer entry points
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status: int, ctx=None) -> None:
    if status != ME_OK:
        detail = ""
        if ctx:
            detail = (lib().me_last_error(ctx) or b"").decode()
        raise MEError(status, detail)
