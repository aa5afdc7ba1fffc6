/*
 * me.h -- C ABI of the MI355X full-search block-matching engine (libme_hip.so).
 *
 * Drop-in boundary for the reference's hot path (souravBhat/MotionEstimation,
 * paths relative to the reference tree):
 *
 *   reference seam                                   replaced by
 *   -----------------------------------------------  ---------------------------------
 *   dispatch region src/cpu/main.c:144-158           me_full_search()
 *     (thpool_init(100) + one findBestBlkMse job       frame level, host planes,
 *      per block + thpool_wait)                        synchronous
 *   findBestBlkMse  src/cpu/main.c:67-82             me_full_search() / me_find_best_blocks()
 *     + findBestMatchMse :39-64 + computeMse :18-36    (per-block calls make no sense on a GPU)
 *   GPU host region src/gpu/main_mse.cu:202-229      me_full_search_device() (HBM-resident,
 *     (H2D, f_findBestMatchBlock<<<>>>, D2H)           stream-ordered)
 *   block list filled for motionCompensatedFrame     me_find_best_blocks() writes the
 *     src/common/utils.c:102-108                       reference's block records
 *
 * Semantics (identical to src/cpu on the same inputs):
 *   - blocks tile the frame in raster order, ceil(W/B) x ceil(H/B), partial
 *     blocks on the right/bottom edges   (src/common/prediction_frame.c:9-23)
 *   - candidates: every top-left whose whole block fits the window
 *     [tl - S, br + S] clamped to the frame   (src/cpu/main.c:53-54, 73-76)
 *   - the first minimum in raster order (y outer, x inner, strict <) wins
 *     (src/cpu/main.c:53-60)
 *   - MV = candidate top-left - block top-left   (src/cpu/main.c:58-59)
 *   - ME_COST_SSD reproduces the reference's float-MSE choice bit for bit:
 *     block_cost = integer SSD of the chosen vector and the reference's score
 *     is (float)block_cost / (float)(w*h) for w*h <= 256; larger blocks are
 *     searched with the reference's float accumulation replayed exactly.
 *   - ME_COST_SAD: same loops and tie rule with |cur - ref| (the reference
 *     has no SAD; parity is against the repo's CPU restatement).
 *   - ME_COST_SSIM: the reference's SSIM search (src/common/ssim.c:3-108,
 *     src/cpu/main_ssim.c:15-29), float arithmetic replayed in its order.
 *
 * Conventions: host buffers are caller-owned; host entry points are
 * synchronous on return.  A context is used by one host thread at a time.
 * Errors are returned, never exit()ed (the reference exits: main.c:134-139).
 */
#ifndef ME_H
#define ME_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ME_API_VERSION 1

typedef enum {
  ME_OK = 0,
  ME_EINVAL = 1,      /* bad argument (sizes, null pointers, block/range limits) */
  ME_ENOMEM = 2,      /* host or device allocation failed */
  ME_EDEVICE = 3,     /* HIP runtime / kernel launch error */
  ME_ECOMM = 4,       /* RCCL error in the multi-device gather */
  ME_EUNSUPPORTED = 5, /* valid request this build cannot serve */
  ME_EIO = 6           /* file missing, short or malformed (me_yuv_* / me_mv_*) */
} me_status;

typedef enum {
  ME_COST_SSD = 0, /* reference parity: float MSE argmin; cost = SSD */
  ME_COST_SAD = 1, /* sum of absolute differences */
  ME_COST_SSIM = 2 /* reference parity with src/common/ssim.c: float SSIM argmax
                      (first strict maximum above 0); cost = the score's float
                      bits; MV (0, 0) and cost 0 where no score is above 0 */
} me_cost;

/* Limits of this build. */
#define ME_MAX_BLOCK 64    /* block_size in [1, 64]  (SSD of 64x64 < 2^32) */
#define ME_MAX_RANGE 1024  /* search_range in [0, 1024] */
/* stride * height < 2^31 bytes per plane (ME_EUNSUPPORTED otherwise). */

typedef struct me_ctx me_ctx;

/* Create a context on n_devices HIP devices (device_ids may be NULL with
 * n_devices <= 1: the current device).  With n_devices > 1 every search is
 * split into macroblock row stripes, one per device, and the per-stripe MV
 * fields are gathered to device_ids[0] with one RCCL ncclGather.  A device id
 * may repeat: repeated ids run their stripes one after another on that device
 * and are gathered by device copies (exercises the stripe path on one GPU). */
me_status me_create(me_ctx** ctx, const int* device_ids, int n_devices);
void me_destroy(me_ctx* ctx);

const char* me_status_str(me_status s);
/* Detail of the last error on this context ("" if none). */
const char* me_last_error(const me_ctx* ctx);
/* Library version string, e.g. "me_hip 1 gfx950". */
const char* me_version(void);

/* Kernel path (process-wide; A/B tests and diagnostics).  Results are
 * identical on every path.
 *   ME_PATH_AUTO: SSD with 16x16 and 8x8 blocks on the matrix cores (i8 MFMA),
 *     everything else on the VALU kernels.  16x16 SSD with S <= 64 runs the
 *     band-walk kernel (each 16-row band's S2 term formed once in LDS for
 *     every block row in flight, no context scratch, ~1.1x the algorithmic
 *     HBM bytes: DESIGN.md) when a launch's strips of block columns fill the
 *     GPU's CUs by themselves (e.g. 16 1080p frames per batched call);
 *     otherwise (single frames, small batches, larger ranges) the prepass +
 *     block-major pair.
 *   ME_PATH_VALU: VALU kernels only.
 *   ME_PATH_MFMA_TILES: 16x16 SSD on the 4x4-block-tile MFMA kernel (the
 *     fallback for rows that are not 16-byte aligned).
 *   ME_PATH_MFMA_LEAN: 16x16 SSD with S <= 64 on the band-walk kernel for
 *     every launch (single frames split into segments of block rows; no
 *     context scratch); a partial bottom block row, or rows the band-walk
 *     kernel cannot take, on the per-workgroup S2 kernel (me_mfma_bmv_kernel).
 *   ME_PATH_MFMA_PREPASS: 16x16 SSD on the S2 prepass + block-major kernel
 *     (5 bytes of context scratch per reference pixel per frame of a batch).
 * The environment variable ME_PATH=auto|valu|tiles|lean|prepass sets the
 * initial value (anything else is ignored with a message on stderr). */
typedef enum {
  ME_PATH_PROCESS = -1,  /* me_ctx_set_kernel_path only: follow the process-wide path */
  ME_PATH_AUTO = 0,
  ME_PATH_VALU = 1,
  ME_PATH_MFMA_TILES = 2,
  ME_PATH_MFMA_LEAN = 3,
  ME_PATH_MFMA_PREPASS = 4
} me_path;
void me_set_kernel_path(me_path path);

/* Per-context kernel path (one host thread per context, as every entry point):
 * the searches of ctx -- planning, scratch and launch, on every device of the
 * context and on the pair pipeline's worker threads -- use `path` (an
 * me_path value) instead of the process-wide one; ME_PATH_PROCESS (the
 * default of a new context) follows me_set_kernel_path / ME_PATH again.
 * ME_EINVAL for an unknown value.  Graphs captured earlier keep the kernels
 * they recorded. */
me_status me_ctx_set_kernel_path(me_ctx* ctx, int path);

/* The kernel family that ran the most recent search launched in this process
 * (any context, any thread -- me_ctx_last_search_path is the per-context one;
 * diagnostics and tests, e.g. that the AUTO path of
 * a 16x16 SSD search is the band-walk kernel).  The matrix-core SSD kernels
 * report the kernel of the frame's full-height block rows. */
typedef enum {
  ME_SEARCH_PATH_NONE = 0,           /* no search launched yet */
  ME_SEARCH_PATH_VALU = 1,           /* SAD and SSD VALU kernels (flow, item, generic) */
  ME_SEARCH_PATH_MFMA_PREPASS = 2,   /* S2 prepass + block-major MFMA kernel */
  ME_SEARCH_PATH_MFMA_BANDWALK = 3,  /* band-walk MFMA kernel (me_band.hip) */
  ME_SEARCH_PATH_MFMA_LEAN = 4,      /* per-workgroup S2 MFMA kernel (bmv) */
  ME_SEARCH_PATH_MFMA_TILES = 5,     /* 4x4-block-tile MFMA kernel */
  ME_SEARCH_PATH_MFMA_8X8 = 6,       /* 8x8-block MFMA kernel */
  ME_SEARCH_PATH_SSIM = 7            /* SSIM kernels */
} me_search_path;
int me_last_search_path(void);
/* The kernel family (me_search_path) of the most recent search launched by
 * ctx on its device devs[device_index] (the index into me_create's device
 * list); ME_SEARCH_PATH_NONE before its first search, -1 for a bad argument.
 * Per context: a search on another context or thread does not change it. */
int me_ctx_last_search_path(const me_ctx* ctx, int device_index);

/* Tiling helpers (src/common/prediction_frame.c:9-11). */
int me_num_blocks(int width, int height, int block_size);
/* Exact number of candidates the search evaluates (reference clamping). */
uint64_t me_candidate_count(int width, int height, int block_size, int search_range);

/* Frame-level search on host Y planes (8-bit, row pitch `stride` >= width).
 * mv_xy: [nblocks][2] int16 (mvx, mvy), block_cost: [nblocks] (may be NULL). */
me_status me_full_search(me_ctx* ctx, const uint8_t* ref, const uint8_t* cur,
                         int width, int height, int stride, int block_size,
                         int search_range, me_cost cost, int16_t* mv_xy,
                         uint32_t* block_cost);

/* Same search on HBM-resident planes of ctx's first device, enqueued on
 * `stream` (a hipStream_t; NULL = the legacy default stream), asynchronous.
 * d_mv_xy / d_block_cost are device arrays of nblocks entries.
 * Searches of one context are ordered by the library: one enqueued on another
 * stream than the previous search waits for it on the GPU (an event recorded
 * on the previous stream at the switch; the host never blocks), so a stream
 * passed here must stay valid until the context's next search is enqueued.
 * After the stream has finished, me_device_check() reports a search whose
 * in-kernel invariant broke (the synchronous entry points check on their own). */
me_status me_full_search_device(me_ctx* ctx, const uint8_t* d_ref,
                                const uint8_t* d_cur, int width, int height,
                                int stride, int block_size, int search_range,
                                me_cost cost, int16_t* d_mv_xy,
                                uint32_t* d_block_cost, void* stream);

/* One row stripe: block rows [block_row_begin, block_row_end).  d_ref holds
 * frame rows starting at ref_row0 and must cover
 *   [max(0, block_row_begin*B - S), min(H, block_row_end*B + S)),
 * d_cur holds frame rows starting at cur_row0 and must cover
 *   [block_row_begin*B, min(H, block_row_end*B)).
 * Outputs hold the stripe's blocks only, raster order.  This is the unit a
 * multi-process (one rank per GPU) caller shards with. */
me_status me_full_search_stripe_device(me_ctx* ctx, const uint8_t* d_ref,
                                       int ref_row0, const uint8_t* d_cur,
                                       int cur_row0, int width, int height,
                                       int stride, int block_size,
                                       int search_range, me_cost cost,
                                       int block_row_begin, int block_row_end,
                                       int16_t* d_mv_xy, uint32_t* d_block_cost,
                                       void* stream);

/* Several stripes (of one frame or of several frames of the same geometry)
 * searched together: each job is what one me_full_search_stripe_device call
 * would take -- its planes with their first resident rows, its block rows and
 * its output records -- and the results are those of one call per job.  The
 * jobs of a call share launches where the kernels allow it, so a batch fills
 * the GPU where one small stripe cannot: the per-rank step of a multi-GPU
 * split over several frames (a rank may hold different row ranges of
 * different frames, balancing its total rows).  Asynchronous on `stream`. */
typedef struct me_stripe_job {
  const uint8_t* d_ref;
  int ref_row0;
  const uint8_t* d_cur;
  int cur_row0;
  int block_row_begin, block_row_end;
  int16_t* d_mv_xy;        /* (block_row_end - block_row_begin) * ceil(W/B) records */
  uint32_t* d_block_cost;  /* may be NULL */
} me_stripe_job;
me_status me_search_stripes_device(me_ctx* ctx, int width, int height, int stride,
                                   int block_size, int search_range, me_cost cost,
                                   const me_stripe_job* jobs, int n_jobs, void* stream);

/* A batch of n_frames same-shaped stripes (or whole frames: block rows
 * [0, nby)): frame f's rows at d_ref + f * ref_frame_stride and
 * d_cur + f * cur_frame_stride bytes (frames must not overlap), its records at
 * d_mv_xy + 2 * f * nblk and d_block_cost + f * nblk, nblk = (block_row_end -
 * block_row_begin) * ceil(W/B).  The equal-stripes case of
 * me_search_stripes_device.  Each plane stack of the batch stays below 2 GiB
 * ((n_frames - 1) * stride + one frame's bytes; ME_EUNSUPPORTED otherwise). */
me_status me_full_search_batch_device(me_ctx* ctx, const uint8_t* d_ref,
                                      size_t ref_frame_stride, int ref_row0,
                                      const uint8_t* d_cur, size_t cur_frame_stride,
                                      int cur_row0, int width, int height, int stride,
                                      int block_size, int search_range, me_cost cost,
                                      int block_row_begin, int block_row_end, int n_frames,
                                      int16_t* d_mv_xy, uint32_t* d_block_cost,
                                      void* stream);

/* Balanced stripe plan: bounds[0..n_shards] block-row boundaries, each stripe
 * carrying about the same search cost.  The cost of a block row is its block
 * count times (3 * (2S+1) + ny) / 4, ny = its exact candidate-row count: the
 * kernels compute a clipped top / bottom block row at nearly the price of an
 * interior one (whole dy chunks, one staged window per tile), so edge rows are
 * discounted by a quarter of their candidate deficit, not all of it. */
me_status me_plan_stripes(int width, int height, int block_size,
                          int search_range, int n_shards, int* bounds);

/* ---- multi-process stripes (one process per GPU) ----
 * The one exchange step of a sharded search, issued from C so a rank's step
 * costs two native calls instead of a Python collective.  Rank 0 calls
 * me_comm_unique_id and sends the ME_COMM_ID_BYTES bytes to the other ranks
 * out of band (e.g. a torch.distributed broadcast); every rank then calls
 * me_comm_init with them (collective: all ranks at once) to build an RCCL
 * communicator on ctx's first device.  No reference counterpart: the
 * reference is single-process. */
#define ME_COMM_ID_BYTES 128
me_status me_comm_unique_id(void* id);
me_status me_comm_init(me_ctx* ctx, const void* id, int n_ranks, int rank);
/* Gather `bytes` from every rank's device buffer d_send into rank 0's d_recv
 * (n_ranks * bytes, rank order; d_recv is ignored on other ranks), enqueued on
 * `stream` (a hipStream_t) after the work already on it; asynchronous. */
me_status me_gather_device(me_ctx* ctx, const void* d_send, size_t bytes, void* d_recv,
                           void* stream);
/* Failure detection for the exchange (the reference checks CUDA
 * errors once, at exit: src/gpu/main_mse.cu:275-276).  Waits at most
 * timeout_ms for the work enqueued so far on `stream` (the rank's searches and
 * gathers) while polling RCCL's asynchronous error (ncclCommGetAsyncError).
 * ME_OK: the stream drained and RCCL reports no error.  ME_ECOMM: RCCL
 * reported an error, or the wait timed out (a peer rank stalled or died); the
 * communicator is then aborted (ncclCommAbort), so this rank's RCCL kernels
 * return and the stream can be synchronised instead of hanging, and every
 * later me_gather_device / me_comm_check on the context fails with ME_ECOMM
 * until me_comm_init builds a new communicator (all ranks, a fresh id).
 * me_last_error names the cause.  The multi-device me_full_search waits the
 * same way (ME_COMM_TIMEOUT_MS) and rebuilds its group after a failure. */
#define ME_COMM_TIMEOUT_MS 60000
me_status me_comm_check(me_ctx* ctx, void* stream, int timeout_ms);

/* ME_EDEVICE if a search kernel of this context reported a broken in-kernel
 * invariant (a bounded wait that expired: the kernel ends instead of hanging
 * the GPU, and that search's MV field is invalid) since the last check; the
 * report is cleared.  Call after the searches' streams have finished.
 * me_full_search, me_find_best_blocks and me_search_pairs check on their own;
 * the word is per device, so such a synchronous call also fails with
 * ME_EDEVICE when an earlier, still unchecked asynchronous search on the
 * device broke its invariant, and the report stays pending for that
 * search's own me_device_check as well. */
me_status me_device_check(me_ctx* ctx);

/* ---- captured steps (hipGraph) ----
 * A per-frame step of device entry points (e.g. a stripe search and its
 * me_gather_device) recorded once and replayed with one launch: the sharded
 * step of a small stripe is bound by host enqueue time, not by the GPU.
 * Counterpart of the reference's per-frame host region (src/gpu/main_mse.cu:202-229).
 *   me_capture_begin(ctx, s); me_full_search_stripe_device(ctx, ..., s);
 *   me_gather_device(ctx, ..., s); me_capture_end(ctx, s, &g);
 *   per frame: me_graph_launch(g, s);
 * `stream` is a created hipStream_t (not NULL).  Run each search once
 * uncaptured first: it sizes the context's scratch, and a captured search that
 * would have to grow it fails with ME_EINVAL.  The captured calls only record;
 * nothing runs until me_graph_launch, which orders the graph after the
 * context's previous search like any search.  A graph whose context scratch
 * was regrown since capture (a larger search ran) is refused (ME_EINVAL).
 * Destroy graphs before their context. */
typedef struct me_graph me_graph;
me_status me_capture_begin(me_ctx* ctx, void* stream);
me_status me_capture_end(me_ctx* ctx, void* stream, me_graph** graph);
me_status me_graph_launch(me_graph* graph, void* stream);
void me_graph_destroy(me_graph* graph);

/* Reference block record, field for field src/common/block.h:6-19 (44 B). */
typedef struct me_ref_block {
  int idx_x, idx_y;
  int top_left_x, top_left_y;
  int bottom_right_x, bottom_right_y;
  int width, height;
  int is_best_match_found;
  int motion_vectorX, motion_vectorY;
} me_ref_block;

/* Adapter for the reference driver: takes its int-widened planes
 * (src/common/utils.c:49-53), searches with ME_COST_SSD and fills
 * motion_vectorX/Y and is_best_match_found = 1 of every block exactly as the
 * thread-pool loop at src/cpu/main.c:144-158 does.  blks must hold the
 * me_num_blocks() records createPredictionFrame produced. */
me_status me_find_best_blocks(me_ctx* ctx, const int* ref_frame,
                              const int* cur_frame, int width, int height,
                              int block_size, int search_range,
                              me_ref_block* blks, int num_blks);

/* ---- consumers of the MV field (src/common/utils.c:94-164) on the GPU ---- */

/* mc[p] = ref[p + mv(block of p)], host planes, synchronous. */
me_status me_motion_compensate(me_ctx* ctx, const uint8_t* ref, int width,
                               int height, int block_size, const int16_t* mv_xy,
                               uint8_t* mc);

/* The reference's 5-plane output [ref, cur, mc, |ref-cur|, |mc-cur|]
 * (src/cpu/main.c:161-168) into out[5*W*H], plus the PSNR of mc vs cur with
 * the reference's MAX = largest pixel rule (src/common/utils.c:137-164). */
me_status me_compensate_planes(me_ctx* ctx, const uint8_t* ref,
                               const uint8_t* cur, int width, int height,
                               int block_size, const int16_t* mv_xy,
                               uint8_t* out5, double* psnr);

/* ---- frame-pair streaming ---- */

/* Pinned (page-locked) host memory.  Frames that live in it are DMAed
 * straight to the device by me_search_pairs; other frames are staged. */
void* me_host_alloc(size_t bytes);
void me_host_free(void* p);

/* Search a list of frame pairs.  frames[0..n_frames) are host Y planes
 * (width x height, row pitch stride); pairs[2*n], pairs[2*n+1] are the
 * (ref, cur) frame indices of pair n, e.g. {0,1, 1,2, 2,3} for a sequence or
 * {0,1, 0,3} for one reference against two currents.  Replaces the
 * reference's one-pair-per-process driver (src/cpu/main.c:109-179): each
 * frame is uploaded once per device, the upload of pair n+1's frames overlaps
 * the search of pair n, and with several context devices the pairs are split
 * into contiguous runs, one per device (no collective: pairs are
 * independent).  Results are those of me_full_search on each pair:
 * mv_xy [n_pairs][nblocks][2], block_cost [n_pairs][nblocks] (may be NULL).
 * Synchronous. */
me_status me_search_pairs(me_ctx* ctx, const uint8_t* const* frames, int n_frames,
                          int width, int height, int stride, int block_size,
                          int search_range, me_cost cost, const int* pairs,
                          int n_pairs, int16_t* mv_xy, uint32_t* block_cost);

/* ---- files: u8 YUV planes and the MV-field format ---- */

/* Raw YUV files as the reference reads and writes them (src/common/utils.c:29-92)
 * but kept in u8 (no int32 widening).  ME_YUV_LUMA: W*H bytes per frame (the
 * reference's frames/ForemanYF*.yuv); ME_YUV_I420: W*H*3/2 bytes per frame,
 * luma first. */
typedef enum { ME_YUV_LUMA = 0, ME_YUV_I420 = 1 } me_yuv_layout;

/* Whole frames in the file, or -1 if it cannot be opened. */
int64_t me_yuv_frame_count(const char* path, int width, int height, me_yuv_layout layout);
/* Luma plane of frame `frame_index` into dst (row pitch dst_stride >= width). */
me_status me_yuv_read_luma(const char* path, int width, int height, me_yuv_layout layout,
                           int frame_index, uint8_t* dst, int dst_stride);
/* Write (append != 0: append) `bytes` bytes, e.g. the 5-plane output of
 * me_compensate_planes (utils.c:75-92 yuvWriteFrame). */
me_status me_yuv_write(const char* path, const uint8_t* data, size_t bytes, int append);

/* MV-field file, little-endian:
 *   header (32 B): "MEMV", u16 version = 1, u16 flags (bit 0: costs present),
 *                  i32 width, height, block_size, search_range, cost, u32 n_pairs
 *   per pair:      i32 ref_index, i32 cur_index,
 *                  nblocks x (i16 mvx, i16 mvy)   raster order
 *                  nblocks x u32 cost             if flags & 1
 * nblocks = me_num_blocks(width, height, block_size). */
typedef struct me_mv_header {
  char magic[4];
  uint16_t version, flags;
  int32_t width, height, block_size, search_range, cost;
  uint32_t n_pairs;
} me_mv_header;

/* pairs: [n_pairs][2] frame indices (NULL: pair n = (n, n+1));
 * block_cost may be NULL (flags bit 0 cleared). */
me_status me_mv_write(const char* path, int width, int height, int block_size,
                      int search_range, me_cost cost, const int* pairs, int n_pairs,
                      const int16_t* mv_xy, const uint32_t* block_cost);
me_status me_mv_read_header(const char* path, me_mv_header* hdr);
/* Read everything; buffers sized from the header (pairs [n_pairs][2],
 * mv_xy [n_pairs][nblocks][2], block_cost [n_pairs][nblocks]); any may be
 * NULL to skip it.  A file without costs leaves block_cost untouched. */
me_status me_mv_read(const char* path, me_mv_header* hdr, int* pairs, int16_t* mv_xy,
                     uint32_t* block_cost);

#ifdef __cplusplus
}
#endif
#endif /* ME_H */
