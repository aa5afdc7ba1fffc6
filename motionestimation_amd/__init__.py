"""motionestimation_amd -- MI355X-native full-search block-matching motion
estimation (drop-in for the hot path of souravBhat/MotionEstimation).

The compute path is libme_hip.so (HIP kernels for gfx950 behind the C ABI of
include/me.h); this package is the host-side mirror of the reference's
interface over that ABI.  There is no CPU fallback.
"""
from ._lib import (ME_COST_SAD, ME_COST_SSD, ME_COST_SSIM, ME_ECOMM, ME_EDEVICE,  # noqa: F401
                   MEError, build)
from .engine import (Engine, candidate_count, num_blocks, pinned_frames,  # noqa: F401
                     last_search_path, plan_stripes, set_kernel_path, version)
from . import io  # noqa: F401
from .reference_api import (Block, PredictionFrame, create_prediction_frame,  # noqa: F401
                            find_best_blk_mse, find_best_blk_ssim, find_best_blks,
                            frame_diff,
                            motion_compensated_frame, output_planes)
