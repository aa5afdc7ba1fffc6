// me_internal.h -- context internals shared by the C-ABI translation units
// (me_api.hip: single-frame and stripe entry points; me_stream.hip: frame-pair
// streaming).  Not installed; include/me.h is the public interface.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "me.h"
#include "me_kernels.h"
#include "me_tuning.h"

namespace me {

class Workers;

struct Dev {
  int id = 0;
  // The context's own stream, created on first use by the host-plane entry
  // points (me_full_search, me_search_pairs, me_compensate_planes, ...): a
  // caller that only uses the device entry points on its own streams never
  // holds it, so a rank of a multi-process split keeps to its hardware queues.
  hipStream_t stream = nullptr;
  hipStream_t copy = nullptr;    // upload stream of the pair pipeline (lazy)
  uint8_t* ref = nullptr;        // frame (or stripe) planes, packed pitch = width
  uint8_t* cur = nullptr;
  size_t frame_cap = 0;
  uint8_t* rec = nullptr;  // [mv int16 x2 | cost u32] x rec_cap blocks
  size_t rec_cap = 0;
  uint8_t* gather = nullptr;  // root only: n_shards * rec bytes
  size_t gather_cap = 0;
  unsigned long long* stats = nullptr;
  uint8_t* out5 = nullptr;
  size_t out_cap = 0;
  uint32_t* sched = nullptr;  // fast-kernel tile counters (self-resetting)
  uint8_t* scratch = nullptr; // MFMA SSD prepass planes (me_mfma.hip), grown on demand
  size_t scratch_cap = 0;
  unsigned long long* mkeys = nullptr;  // MFMA SSD merge keys (~0) and tile counters (0):
  uint32_t* mcnt = nullptr;             //   initialised on allocation, self-resetting after
  size_t merge_cap = 0;                 //   (tiles)
  // The counters, merge keys and scratch above serve one search at a time:
  // a search issued on another stream than the previous one first waits for
  // it (launch_ordered): search_ev is recorded on the previous search's stream
  // at the switch and the new stream waits for it (no host block, no event
  // per search).  Searches captured into a graph (me_capture_begin) are not
  // executed at capture: me_graph_launch orders the graph the same way.
  hipEvent_t search_ev = nullptr;
  hipStream_t search_stream = nullptr;
  bool searched = false;
  // Frame-pair pipeline (me_stream.hip), kept across calls.
  std::vector<uint8_t*> slots;        // device frames, slot_bytes each
  std::vector<uint8_t*> slot_chunks;  // their allocations: kSlotChunk adjacent slots each
  std::vector<uint8_t*> slot_spare;   // slots of the last chunk not handed out yet
  size_t slot_bytes = 0;
  uint8_t* stage[2] = {nullptr, nullptr};  // pinned staging for pageable frames
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  size_t stage_bytes = 0;
  Workers* stage_pool = nullptr;  // helper threads of the staging copy (run_pairs)
  // One event pair per batch of pairs (ring by batch index): the batch's uploads
  // done (copy stream; the compute stream waits on it once) and its search done
  // (compute stream; bounds the host's run-ahead and guards slot reuse).
  hipEvent_t upl_ev[16] = {};
  hipEvent_t batch_ev[16] = {};
  uint8_t* pair_out = nullptr;  // [pairs][nblocks] mv records, then [pairs][nblocks] costs
  size_t pair_out_cap = 0;
  // Records leave per batch, overlapped with the later batches' searches: the
  // copy stream (or, tuning build, a stream of their own) waits for the
  // batch's search and copies its records into pinned `bounce` (pair_out's
  // layout); the host moves them to the caller's arrays while it would
  // otherwise wait for the GPU.
  hipStream_t d2h = nullptr;
  hipEvent_t d2h_ev[16] = {};
  uint8_t* bounce = nullptr;
  size_t bounce_cap = 0;
  // An invariant report that a synchronous entry point read (and cleared on
  // the device) on behalf of earlier asynchronous searches: me_device_check
  // still reports it once (device_status sets it, me_device_check clears it).
  uint32_t err_pending = 0;
  // An asynchronous search (a device entry point or a graph launch on a
  // caller's stream) was enqueued since the last me_device_check: only then
  // may the invariant word a synchronous call reads belong to another search.
  bool async_unchecked = false;
};

// Persistent host workers, one per context device (multi-device searches and
// pair runs): started on first use, joined by me_destroy.  run(n, fn) calls
// fn(i) on worker i for i < n and returns when all have finished; one caller
// at a time (a context is used by one host thread at a time, include/me.h).
class Workers {
 public:
  explicit Workers(int n);
  ~Workers();
  int size() const { return (int)th_.size(); }
  void run(int n, const std::function<void(int)>& fn);
  // fn(0) on the calling thread, fn(1 .. n - 1) on workers 0 .. n - 2
  void run_split(int n, const std::function<void(int)>& fn);

 private:
  void loop(int i);
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable go_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  unsigned long long gen_ = 0;
  int n_ = 0, off_ = 0, pending_ = 0;
  bool stop_ = false;
};

// The context's workers, created with one thread per device on first use
// (nullptr if a thread could not be started).
Workers* workers(me_ctx* c);

// Wait, bounded, for the work enqueued so far on stream s of device d (one
// that ends in RCCL collectives on `comm`), polling the stream and the
// communicator's asynchronous error.  ME_OK when the stream drained;
// ME_ECOMM when RCCL reported an error or timeout_ms passed (a peer stalled or
// died): the caller aborts the communicator.  ev: a scratch event of d.
me_status wait_comm(me_ctx* c, hipStream_t s, hipEvent_t ev, ncclComm_t comm, int timeout_ms);

// Free the pair pipeline's buffers and events of one device (me_destroy).
void release_pipeline(Dev& d);

me_status fail(me_ctx* c, me_status s, const char* fmt, ...);
// Create d's own stream if it does not exist yet (device d must be current).
me_status own_stream(me_ctx* c, Dev& d);
me_status grow(me_ctx* c, void** p, size_t* cap, size_t need);
me_status check_args(me_ctx* c, const void* ref, const void* cur, int width, int height,
                     int stride, int blk, int range, int cost, const void* mv);
SearchArgs make_args(const uint8_t* ref, int ref_row0, const uint8_t* cur, int cur_row0,
                     int width, int height, int stride, int blk, int range, int cost, int r0,
                     int r1, int16_t* mv, uint32_t* cst);

// Point p at d's search scratch, growing it to what p's search needs.  A
// device's scratch serves one search at a time: launch searches that use it
// with launch_ordered.
// cap: the launch is being captured (me_capture_begin): growing the scratch
// then fails with ME_EINVAL (a graph must not hold buffers a later search frees).
// batch > 1: scratch for that many equal-geometry jobs in shared launches
// (mfma_batch_scratch), else for one search
me_status attach_scratch(me_ctx* c, Dev& d, SearchArgs& p, bool cap = false, int batch = 1);

// Launch p (scratch attached) on stream s after every earlier search of d:
// a search arriving on a different stream than the previous one first waits
// for that search's end event.  A failed launch re-zeroes the self-resetting
// tile counters and merge buffers (a partly run kernel may have left them
// dirty) before returning ME_EDEVICE.
me_status launch_ordered(me_ctx* c, Dev& d, SearchArgs& p, hipStream_t s);

// The same for a job table (launch_jobs): jobs share base's geometry, cost and
// scratch (attach_scratch(base, cap, n) for equal jobs).  cap: being captured
// (no ordering, no state change).
me_status launch_jobs_ordered(me_ctx* c, Dev& d, const SearchArgs& base, const SearchJob* jobs,
                              int n, hipStream_t s, bool cap = false);

// Order stream s after the device's previous search (a stream switch) and
// make s the device's search stream; `launch` then enqueues on s.
me_status order_on(me_ctx* c, Dev& d, hipStream_t s);

// True while s is being captured into a graph (me_capture_begin).
bool capturing(hipStream_t s);

// Read and clear the device's in-kernel invariant word (sched[SCHED_ERR])
// after the work on stream s: ME_EDEVICE if a kernel reported a broken
// invariant (a bounded wait that expired), ME_OK otherwise.  Synchronises s.
me_status device_status(me_ctx* c, Dev& d, hipStream_t s);

// Pinned host ranges handed out by me_host_alloc (the pair pipeline DMAs
// straight from them instead of staging).
bool host_range_pinned(const void* p, size_t bytes);

}  // namespace me

struct me_ctx {
  std::vector<me::Dev> devs;
  bool distinct = true;
  ncclComm_t* comms = nullptr;
  ncclComm_t rank_comm = nullptr;  // me_comm_init: one rank of a multi-process group
  int comm_ranks = 0, comm_rank = -1;
  bool comm_aborted = false;       // me_comm_check aborted rank_comm (failure detected)
  hipEvent_t comm_ev = nullptr;    // me_comm_check's marker on the checked stream
  me::Workers* pool = nullptr;     // me::workers(): persistent per-device host threads
  // me_ctx_set_kernel_path: this context's kernel path code (me_tuning.h),
  // -1 = the process-wide one; last_path[i]: ME_SEARCH_PATH_* of the latest
  // search launched on devs[i] (me_ctx_last_search_path)
  int path = -1;
  std::vector<std::atomic<int>> last_path;
  // A per-device error context of a multi-device call (its worker's failure
  // message) points at the context the call is for: the kernel path and the
  // last-path slots are that context's.
  me_ctx* owner = nullptr;
  char err[512] = {0};
};

namespace me {
// The last-path slot of device d of the context c serves (nullptr if d is not
// one of its devices).
inline std::atomic<int>* ctx_last_slot(me_ctx* c, Dev& d) {
  const ptrdiff_t i = &d - c->devs.data();
  return i >= 0 && (size_t)i < c->last_path.size() ? &c->last_path[(size_t)i] : nullptr;
}
}  // namespace me

#define ME_CTX_PATH_SCOPE(c, d)                                  \
  me_ctx* const me_path_ctx_ = (c)->owner ? (c)->owner : (c);    \
  me::PathScope me_path_scope_(me_path_ctx_->path, me::ctx_last_slot(me_path_ctx_, (d)))

#define HIPCHK(ctx, x)                                                                 \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return me::fail(ctx, ME_EDEVICE, "%s:%d %s: %s", __FILE__, __LINE__, #x,         \
                      hipGetErrorString(e_));                                          \
  } while (0)

#define NCCLCHK(ctx, x)                                                                \
  do {                                                                                 \
    ncclResult_t r_ = (x);                                                             \
    if (r_ != ncclSuccess)                                                             \
      return me::fail(ctx, ME_ECOMM, "%s:%d %s: %s", __FILE__, __LINE__, #x,           \
                      ncclGetErrorString(r_));                                         \
  } while (0)
