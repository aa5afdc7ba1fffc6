// me_kernels.h -- device-side launch interface (internal to libme_hip.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace me {

enum { COST_SSD = 0, COST_SAD = 1, COST_SSIM = 2 };

constexpr int GENERIC_THREADS = 256;
constexpr int GENERIC_LDS_BUDGET = 60 * 1024;
constexpr int QSAD_LDS_BUDGET = 40 * 1024;  // 4 workgroups per CU (160 KB LDS)
// sched holds SCHED_WORDS u32: [0, 16) the item kernel's 8 two-ended band
// counters (u64: owner claims in the low half, thieves in the high half),
// [SCHED_ARRIVE] its arrivals (the last workgroup out re-zeroes [0, 17)),
// [SCHED_ERR]: a kernel whose bounded wait expired sets it (the host reads and
// clears it: device_status, me_device_check).
constexpr int SCHED_WORDS = 32;
constexpr int SCHED_ARRIVE = 16;
constexpr int SCHED_ERR = 31;

// One search launch: block rows [block_row_begin, block_row_end) of a
// width x height frame.  ref / cur point at frame rows ref_row0 / cur_row0.
// Outputs are indexed (block row - block_row_begin) * nbx + block column.
struct SearchArgs {
  const uint8_t* ref;
  const uint8_t* cur;
  int ref_row0, cur_row0;
  int width, height, stride;
  int blk, range;
  int nbx;
  int block_row_begin, block_row_end;
  int cost_kind;
  int16_t* mv;
  uint32_t* cost;
  uint32_t ref_bytes;  // readable bytes from ref (buffer range check), and from cur
  uint32_t cur_bytes;
  uint32_t* sched;     // SCHED_WORDS u32 (layout above), zeroed between launches; or null
  uint8_t* scratch;    // device scratch of the MFMA SSD path (mfma_ssd_scratch bytes) or null
  size_t scratch_bytes;
  // MFMA SSD cross-workgroup merge (self-resetting): 16 keys (~0) per tile and
  // one arrival counter (0) per tile, merge_tiles tiles; or null
  unsigned long long* mkeys;
  uint32_t* mcnt;
  size_t merge_tiles;
};

// Write block `out`'s MV from a merged 64-bit key (cost << 32 | (dy + 32768)
// << 16 | (dx + 32768)): one 4-byte store of the (mvx, mvy) int16 pair when the
// records are 4-byte aligned, else two 2-byte stores.  (8K 8x8 WRITE_SIZE reads
// 2x the record bytes either way: a tile's 8 blocks store 32 contiguous bytes
// per array, below the 64-byte write granule the counter appears to tally.)
__device__ __forceinline__ void store_mv(int16_t* mv, int out, unsigned long long kk) {
  if (((uintptr_t)mv & 3) == 0) {
    reinterpret_cast<uint32_t*>(mv)[out] = (uint32_t)kk ^ 0x80008000u;
  } else {
    mv[2 * out] = (int16_t)((int)(kk & 0xFFFF) - 32768);
    mv[2 * out + 1] = (int16_t)((int)((kk >> 16) & 0xFFFF) - 32768);
  }
}

struct QsadGeom {
  int tb;          // blocks per workgroup
  int rows_alloc;  // LDS tile rows (chunks*K + B - 1)
  int row0;        // first block row of the launch
  int nrows;       // block rows in the launch
  int groups;      // 4-wide dx groups per block
  int chunks;      // K-row dy chunks
  int cpp;         // dy chunks per LDS pass
  int pitch;       // bytes per LDS tile row (multiple of 16)
  int tile_bytes;  // rows_alloc * pitch
  uint32_t pitch_magic;  // umulhi(d, pitch_magic) == d / pitch on the staged range
  uint32_t magic_groups; // umulhi(t, magic_groups) == t / groups on an item's tasks
  int threads;     // workgroup size
  int lds;         // dynamic LDS bytes
  int wg_per_row;  // workgroups per block row
  uint32_t magic_wpr;  // umulhi(t, magic_wpr) == t / wg_per_row for every tile index of
                       // the planned rows (host-checked; 0: divide)
  uint32_t magic_tb;   // 0xFFFFFFFF / tb + 1: an item's / nb magic when nb == tb
  int strip_w;     // > 0: tiles run in vertical strips of strip_w tile columns, each
                   // strip top to bottom (wide frames: an XCD's L2 keeps the strip's
                   // window rows while the tile rows that read them pass)
  int nbx_full;    // full-width blocks per row
  int aligned;     // 4-byte aligned global rows
  int tile16;      // ref tile staged in 16-byte granules (X0, width, rows 16-byte aligned)
  int fold;        // SAD, S % 4 == 0: groups = S/2 cover dx in [-S, S-1]; the dx = +S
                   // column is spread over lanes gi < K, one v_sad_u8 candidate each
  int dyn_tiles;   // dynamic tile pulls when tiles >= dyn_tiles * workgroups (0: never)
  int pull_ahead;  // dynamic: tile ti + pull_ahead is claimed when tile ti starts (1 or 2)
  int flow_slots;  // me_flow_kernel: LDS ring slots (0: the persistent item kernel)
  int prio;        // waves issuing staging raise their issue priority (s_setprio) meanwhile
  int fair;        // me_flow_kernel: lo | hi << 8 | mode << 16 (0: off): a wave whose
                   // wave-task others have overtaken by >= lo / hi pulls raises its
                   // issue priority to 1 / 2 (checked every 4 rows; 8 / 16 by
                   // default) in launches with slot refills (mode 1)
};

// A search job: block rows [r0, r1) of one frame (or row stripe), its planes
// (ref / cur hold frame rows from ref_row0 / cur_row0, as in SearchArgs) and
// its records (indexed from r0).  Jobs of one launch share the frame geometry.
struct SearchJob {
  const uint8_t* ref;
  int ref_row0;
  const uint8_t* cur;
  int cur_row0;
  int r0, r1;
  int16_t* mv;
  uint32_t* cost;
};

// The flow kernel's job table (kernel argument): job j owns launch tiles
// [tile_pre[j], tile_pre[j + 1]).  A batch of frames or stripes (the per-rank
// step of a multi-GPU split) fills the GPU in one launch.
constexpr int MAX_JOBS = 32;
struct FlowJobs {
  int n;
  int tile_pre[MAX_JOBS + 1];
  int r0[MAX_JOBS];
  int ref_row0[MAX_JOBS], cur_row0[MAX_JOBS];
  uint32_t ref_bytes[MAX_JOBS], cur_bytes[MAX_JOBS];
  const uint8_t* ref[MAX_JOBS];
  const uint8_t* cur[MAX_JOBS];
  int16_t* mv[MAX_JOBS];
  uint32_t* cost[MAX_JOBS];
};

// Equal-geometry SSD searches of one matrix-core launch pair (prepass + main
// kernel): frames of one size and the same block rows.  Job j's planes and
// records are its own, its prepass planes sit at scratch + j * scratch_stride.
// A single search is the one-job table of its own pointers.
struct MfmaJobs {
  int n;
  int wgs;                // main-kernel workgroups per job
  size_t scratch_stride;  // bytes between consecutive jobs' prepass planes
  const uint8_t* ref[MAX_JOBS];
  const uint8_t* cur[MAX_JOBS];
  int16_t* mv[MAX_JOBS];
  uint32_t* cost[MAX_JOBS];
};

// Search every job (geometry, cost and scratch from base): SAD jobs the flow
// kernel takes share one launch (up to MAX_JOBS jobs), VALU jobs of the item
// kernel likewise, everything else runs job by job through launch_search.
hipError_t launch_jobs(const SearchArgs& base, const SearchJob* jobs, int n, hipStream_t stream);

// Matrix-core SSD path (me_mfma.hip): B = 16, full-height rows [row0, row0 +
// nrows) x full-width columns [0, nbx); 4x4-block tiles.
struct MfmaGeom {
  int row0, nrows, nbx;
  int tiles_x, tiles_y;
  int ngx;               // 64-position groups per tile
  int ngxw;              // groups per workgroup (16x16 tiles: 1 or 2, 4 waves each; 8x8: all, in turn)
  int km;                // candidate rows per chunk L = 13 + 16 km
  int bm, bm_wpr, bm_lp; // block-major kernel (16x16, S <= 192); workgroups per block row; window pitch
  int bmv;               // block-major kernel forming S2 itself (S <= 64): no prepass, no scratch
  int bmv_r;             // ... its block rows per workgroup (1 or 2)
  int lds;               // dynamic LDS bytes
  int hb, hb_row;        // partial bottom block row: height hb, block row index (-1: none)
  int ya0, rp_rows;      // frame rows [ya0, ya0 + rp_rows) of the prepass planes
  int rows_alloc;        // plane rows written (rp_rows + read slack)
  int pitch;             // row pitch of the planes (entries)
  int s2h_row0;          // first s2h row the kernel reads
  uint32_t rp_bytes, s2_bytes;  // buffer ranges (s2_bytes spans s2 and s2h)
  uint32_t s2h_off;      // byte offset of s2h from s2
  size_t scratch_bytes;
  int8_t* rp;            // ref ^ 0x80
  int* s2;               // 16x16 box sums of (ref - 127)^2
  int* s2h;              // hb x 16 box sums (partial bottom row only)
  unsigned long long* mkeys;  // per tile 16 merge keys (~0 between launches)
  uint32_t* mcnt;        // per tile arrival counters (0 between launches)
  // Band-walk kernel (me_band.hip, 16x16, the default for S <= 64): a
  // workgroup walks a strip of block columns down a segment of block rows,
  // forming each 16-row band's S2 once in LDS for every block row in flight.
  int bw;                // 1: this plan runs on it (full-height rows [row0, row0 + nrows))
  int bw_wpc, bw_ns;     // waves per block column (row classes), ring slots per wave
  int bw_nsw, bw_pw;     // searcher and producer waves per workgroup
  int bw_cols;           // block columns per strip (bw_nsw / bw_wpc)
  int bw_strips;         // strips per job
  int bw_seg_rows;       // block rows per workgroup (segment)
  int bw_segs;           // segments per job
  int bw_xt;             // per-XCD tail split (bw_cx CUs per XCD): workgroup decode in bw_item()
  int bw_cx;
  int bw_lp, bw_pp;      // window row pitch (bytes), P0 plane row pitch (ints)
  int bw_abl;            // tuning build only: ablation bits (ME_BW_ABL), 0 in the product
  int bw_hb;             // S2 planes of a partial bottom row run by the band-walk kernel (0: by bmv)
};
size_t mfma_merge_tiles(const SearchArgs& p);  // tiles the merge buffers must cover
bool plan_mfma_ssd(const SearchArgs& p, MfmaGeom* g);
hipError_t launch_mfma_ssd(const SearchArgs& p, const MfmaGeom& g, hipStream_t stream);
size_t mfma_ssd_scratch(const SearchArgs& p);  // 0: path not applicable
// Scratch for n equal-geometry jobs of p's shape in batched launches (the
// block-major kernel; at most MAX_JOBS per launch, capped near 1 GiB), or
// mfma_ssd_scratch(p) when they would run one by one.
size_t mfma_batch_scratch(const SearchArgs& p, int n);
// Equal-geometry SSD jobs on the block-major kernel, in launches of as many
// jobs as the scratch holds.  False (nothing launched): not applicable.
bool launch_mfma_jobs(const SearchArgs& base, const SearchJob* jobs, int n, hipStream_t stream,
                      hipError_t* err);
// Band-walk kernel (me_band.hip): plan the full-height rows of p into g (g's
// common fields already set by plan_mfma_ssd), and launch every job of jb.
bool plan_bw(const SearchArgs& p, MfmaGeom* g, int jobs);
// The band-walk plan g (plan_bw) for `jobs` jobs per launch runs in one
// round of workgroups (every segment of every strip resident at once).
bool bw_one_round(const MfmaGeom& g, int jobs);
hipError_t launch_bw(const SearchArgs& p, const MfmaGeom& g, const MfmaJobs& jb, hipStream_t stream);
// Tiles of cross-workgroup merge buffers (mkeys: 16 u64 keys each, ~0; mcnt:
// one u32 counter each, 0) the search of p needs (the MFMA SSD kernels).
size_t merge_tiles_needed(const SearchArgs& p);
bool mfma_disabled();

hipError_t launch_search(const SearchArgs& p, hipStream_t stream, int* used_fast);
// Records the kernel family of a search being launched (ME_SEARCH_PATH_*):
// process-wide (me_last_search_path) and, inside a PathScope, for the
// context device the search runs on (me_ctx_last_search_path).
void note_path(int path);
int last_path();
// Raise fn's dynamic-LDS limit to lds (> 64 KB) on the current device, once
// per (kernel, device, larger size): process-wide cache, thread-safe.
hipError_t lds_attr(const void* fn, int lds);
hipError_t launch_generic(const SearchArgs& p, int bx0, int nbx_range, int row0, int nrows,
                          hipStream_t stream);
bool plan_fast(const SearchArgs& p, QsadGeom* g, int* k_out);

// SSIM-cost search (me_ssim.hip): every block of rows [block_row_begin, block_row_end).
hipError_t launch_ssim(const SearchArgs& p, hipStream_t stream);
// Scratch bytes of the SSIM search's patch-statistics plane (0: not applicable).
size_t ssim_scratch(const SearchArgs& p);

// Consumers of the MV field (me_post.hip).
hipError_t launch_compensate(const uint8_t* ref, const uint8_t* cur, int width, int height,
                             int blk, const int16_t* mv, uint8_t* out5, int write_planes,
                             unsigned long long* stats, hipStream_t stream);

}  // namespace me
