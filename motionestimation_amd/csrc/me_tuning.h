// me_tuning.h -- planner overrides for the tuning tools (internal).
//
// The default build (libme_hip.so) reads no environment beyond the documented
// ME_PATH (include/me.h): tuning() returns the automatic settings.  The
// diagnostic build libme_hip_tune.so (csrc/Makefile `tune`, -DME_TUNING in
// me_api.hip only) parses the overrides below once per process, thread-safely,
// and rejects malformed values with a message on stderr (the automatic setting
// stays).  tools/plan_sweep.py, tools/dyn_sweep.sh and tools/dbg/* select it
// with ME_HIP_LIB=libme_hip_tune.so.
#pragma once

#include <atomic>

namespace me {

struct Tuning {
  // ME_PLAN="K,tb,cpp,threads[,fold]": fast-kernel plan (0 = free; fold -1 = free)
  int plan_k = 0, plan_tb = 0, plan_cpp = 0, plan_threads = 0, plan_fold = -1;
  int dyn = -1;           // ME_DYN: tiles per workgroup for dynamic pulls (-1 = automatic)
  int mfma_bm = 2;        // ME_MFMA_BM=0|1: block-major SSD kernel off / on (2 = automatic)
  int mfma_km = 0;        // ME_MFMA_KM=2|3: 8x8/tile kernel chunk length (0 = automatic)
  int mfma_ngxw = 0;      // ME_MFMA_NGXW=1|2: column groups per workgroup (0 = automatic)
  int stream_cool = 0;    // ME_STREAM_COOL=1..64: cooling frame slots (0 = automatic)
  int stream_ahead = 0;   // ME_STREAM_AHEAD=1..9: host run-ahead (9: unbounded; 0 = automatic)
  int stream_batch = 0;   // ME_STREAM_BATCH=1..32: pairs per search launch after the ramp (0 = automatic)
  int stream_d2h = 0;     // ME_STREAM_D2H=1: pair records download on a stream of their own
  int stream_cpy = 0;     // ME_STREAM_CPY=1..16: threads of a pageable frame's staging copy (0 = 4)
  int stream_ramp = -1;   // ME_STREAM_RAMP=0: no ramp, every launch ME_STREAM_BATCH pairs (-1 = ramp)
  int stream_grow = 0;    // ME_STREAM_GROW=1..20: ramp growth per batch in tenths (0 = 5: 1.5x)
  int stream_upl = 0;     // ME_STREAM_UPL=1..3: batches the uploads run ahead of the searches (0 = 1)
  int flow = -1;          // ME_FLOW=0|1: SAD flow kernel off / allowed (-1 = automatic)
  int flow_slots = 0;     // ME_FLOW_SLOTS=2..16: flow kernel LDS ring slots (0 = automatic)
  int prio = -1;          // ME_PRIO=0|1: staging waves raise their issue priority (-1 = automatic: on)
  int fair = -1;          // ME_FAIR=0..3: flow-kernel waves behind the pull counter raise their priority: 0 off, 1 in launches
                          // with refills (automatic), 2 on items whose slot gets a refill, 3 always
  int fair_lo = 8, fair_hi = 16;  // ME_FAIR_T=lo,hi: the lags (pulls) that raise a wave to priority 1 / 2
  int flow_one = -1;      // ME_FLOW_ONE=0|1: a batch's flow jobs in launches of one ring / in one launch (-1 = automatic: one)
  int mfma_s2k = -1;      // ME_MFMA_S2K=0|1: 16x16 SSD, S <= 64: S2 from the prepass plane / formed in
                          // the workgroup (-1 = automatic: the kernel path, ME_PATH_MFMA_LEAN)
  int mfma_s2r = 0;       // ME_MFMA_S2R=1|2: lean path block rows per workgroup (0 = automatic: 2 from S = 48)
  int mfma_batch = -1;    // ME_MFMA_BATCH=0|1: equal SSD jobs share matrix-core launches (-1 = automatic: on)
  int item_batch = -1;    // ME_ITEM_BATCH=0: item-kernel jobs launch one by one (diagnostic)
  int ahead = -1;         // ME_AHEAD=1|2: item-kernel tiles claimed ahead (-1 = automatic)
  int strip = -1;         // ME_STRIP=0..64: item-kernel tile strips (0 = row-major; -1 = automatic)
  int bw = -1;            // ME_BW=0|1: 16x16 SSD band-walk kernel off / on where it applies (-1 = automatic: on)
  int bw_hb = -1;         // ME_BW_HB=0: a partial bottom row on the lean kernel, not in the band walk
  int fast_res = 0;       // ME_FAST_RES=1..32: item-kernel workgroups per CU at most (0 = what fits)
  int bw_xt = -1;         // ME_BW_XT=0: uniform segments, no per-XCD tail split
  int bw_seg = 0;         // ME_BW_SEG=1..4096: band-walk block rows per workgroup (0 = automatic)
  int bw_abl = 0;         // ME_BW_ABL=0..1023: band-walk ablations, timing only (results invalid):
                          // 1 no production (nor XOR-ed window), 2 no tiles, 4 no row entries,
                          // 64 no key epilogue, 128 no B-fragment reads in the tiles, 256 the
                          // MFMAs of ring slot 0 only;
                          // variants (results valid): 16 producer waves at raised priority,
                          // 32 producer waves at raised priority for the first ring of bands
};

const Tuning& tuning();

// Kernel path: 0 automatic, 1 VALU kernels only, 2 the 4x4-block-tile MFMA
// kernel for 16x16 SSD (no block-major kernel), 3 band-walk for every 16x16
// SSD launch with S <= 64 (ME_PATH_MFMA_LEAN), 4 the prepass + block-major
// pair (ME_PATH_MFMA_PREPASS).  The process-wide code (me_set_kernel_path /
// ME_PATH) applies unless a PathScope of a context with its own path
// (me_ctx_set_kernel_path) is active on the calling thread.  Atomic: read by
// planner threads.
int kernel_path();
void set_kernel_path_code(int v);
int path_code_of(int me_path_value);  // ME_PATH_* -> code above (-1 if invalid)

// While alive on a thread: kernel_path() returns `path` when it is >= 0, and
// note_path() also stores into *last (the context device's last search path).
// Set around the planning and launch of a context's search (attach_scratch,
// launch_ordered, launch_jobs_ordered); nests.
struct PathScope {
  PathScope(int path, std::atomic<int>* last);
  ~PathScope();
  PathScope(const PathScope&) = delete;
  PathScope& operator=(const PathScope&) = delete;
  int prev_path;
  std::atomic<int>* prev_last;
};

}  // namespace me
