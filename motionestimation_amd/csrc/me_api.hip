// me_api.hip -- C ABI of libme_hip.so (declared in include/me.h).
//
// Host side of the engine: argument checking (status codes, never exit()),
// device buffers owned by the context, the stripe planner, and the
// multi-device path (row stripes + one RCCL ncclGather of the per-stripe MV
// records to the first device).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <new>
#include <thread>
#include <vector>

#include "me_internal.h"

using me::Dev;

namespace me {

// ------------------------------------------------------------ tuning knobs
#ifdef ME_TUNING
// Diagnostic build only (libme_hip_tune.so): validated environment overrides.
static bool env_int(const char* name, int lo, int hi, int* out) {
  const char* e = getenv(name);
  if (!e || !*e) return false;
  char* end = nullptr;
  const long v = strtol(e, &end, 10);
  if (*end || v < lo || v > hi) {
    fprintf(stderr, "me_hip: ignoring %s=%s (expected an integer in [%d, %d])\n", name, e, lo, hi);
    return false;
  }
  *out = (int)v;
  return true;
}

static Tuning read_tuning() {
  Tuning t;
  if (const char* e = getenv("ME_PLAN")) {
    int v[5] = {0, 0, 0, 0, -1};
    const int n = sscanf(e, "%d,%d,%d,%d,%d", &v[0], &v[1], &v[2], &v[3], &v[4]);
    const bool ok = n >= 4 && (v[0] == 0 || v[0] == 4 || v[0] == 5 || v[0] == 8 || v[0] == 11 || v[0] == 13 || v[0] == 26) &&
                    v[1] >= 0 && v[1] <= 16 && v[2] >= 0 && v[2] <= 64 &&
                    (v[3] == 0 || (v[3] >= 64 && v[3] <= 1024 && v[3] % 64 == 0)) &&
                    v[4] >= -1 && v[4] <= 1;
    if (ok) {
      t.plan_k = v[0]; t.plan_tb = v[1]; t.plan_cpp = v[2]; t.plan_threads = v[3]; t.plan_fold = v[4];
    } else {
      fprintf(stderr, "me_hip: ignoring ME_PLAN=%s (K in {0,4,5,8,11,13,26}, tb 0..16, cpp 0..64, "
                      "threads 0 or 64..1024 step 64, fold -1..1)\n", e);
    }
  }
  env_int("ME_DYN", 0, 1 << 20, &t.dyn);
  env_int("ME_MFMA_BM", 0, 1, &t.mfma_bm);
  env_int("ME_MFMA_KM", 2, 3, &t.mfma_km);
  env_int("ME_MFMA_NGXW", 1, 2, &t.mfma_ngxw);
  env_int("ME_STREAM_COOL", 1, 64, &t.stream_cool);
  env_int("ME_STREAM_AHEAD", 1, 9, &t.stream_ahead);
  env_int("ME_STREAM_BATCH", 1, 32, &t.stream_batch);
  env_int("ME_STREAM_RAMP", 0, 1, &t.stream_ramp);
  env_int("ME_STREAM_UPL", 1, 3, &t.stream_upl);
  env_int("ME_STREAM_GROW", 1, 20, &t.stream_grow);
  env_int("ME_STREAM_D2H", 0, 1, &t.stream_d2h);
  env_int("ME_STREAM_CPY", 1, 16, &t.stream_cpy);
  env_int("ME_FLOW", 0, 1, &t.flow);
  env_int("ME_FLOW_SLOTS", 2, 16, &t.flow_slots);
  env_int("ME_PRIO", 0, 1, &t.prio);
  env_int("ME_STRIP", 0, 64, &t.strip);
  env_int("ME_FAST_RES", 1, 32, &t.fast_res);
  env_int("ME_AHEAD", 1, 2, &t.ahead);
  env_int("ME_ITEM_BATCH", 0, 1, &t.item_batch);
  env_int("ME_FAIR", 0, 3, &t.fair);
  env_int("ME_FLOW_ONE", 0, 1, &t.flow_one);
  env_int("ME_MFMA_BATCH", 0, 1, &t.mfma_batch);
  env_int("ME_MFMA_S2K", 0, 1, &t.mfma_s2k);
  env_int("ME_MFMA_S2R", 1, 2, &t.mfma_s2r);
  env_int("ME_BW", 0, 1, &t.bw);
  env_int("ME_BW_SEG", 1, 4096, &t.bw_seg);
  env_int("ME_BW_HB", 0, 1, &t.bw_hb);
  env_int("ME_BW_XT", 0, 1, &t.bw_xt);
  env_int("ME_BW_ABL", 0, 1023, &t.bw_abl);
  if (const char* e = getenv("ME_FAIR_T")) {
    int lo = 0, hi = 0;
    if (sscanf(e, "%d,%d", &lo, &hi) == 2 && lo >= 1 && lo <= hi && hi <= 255) {
      t.fair_lo = lo;
      t.fair_hi = hi;
    } else {
      fprintf(stderr, "me_hip: ignoring ME_FAIR_T=%s (lo,hi with 1 <= lo <= hi <= 255)\n", e);
    }
  }
  return t;
}
const Tuning& tuning() {
  static const Tuning t = read_tuning();  // once, thread-safe (C++11 static init)
  return t;
}
#else
const Tuning& tuning() {
  static const Tuning t;  // automatic settings; the product reads no tuning knobs
  return t;
}
#endif

// ME_PATH (include/me.h): initial kernel path; me_set_kernel_path overrides it.
static int initial_path() {
  const char* e = getenv("ME_PATH");
  if (!e || !*e || !strcmp(e, "auto")) return 0;
  if (!strcmp(e, "valu")) return 1;
  if (!strcmp(e, "tiles")) return 2;
  if (!strcmp(e, "lean")) return 3;
  if (!strcmp(e, "prepass")) return 4;
  fprintf(stderr, "me_hip: ignoring ME_PATH=%s (auto | valu | tiles | lean | prepass)\n", e);
  return 0;
}
static std::atomic<int>& path_code() {
  static std::atomic<int> v{initial_path()};
  return v;
}
static thread_local int tl_path = -1;
static thread_local std::atomic<int>* tl_last = nullptr;
int kernel_path() { return tl_path >= 0 ? tl_path : path_code().load(std::memory_order_relaxed); }
void set_kernel_path_code(int v) { path_code().store(v, std::memory_order_relaxed); }
int path_code_of(int v) {
  switch (v) {
    case ME_PATH_AUTO: return 0;
    case ME_PATH_VALU: return 1;
    case ME_PATH_MFMA_TILES: return 2;
    case ME_PATH_MFMA_LEAN: return 3;
    case ME_PATH_MFMA_PREPASS: return 4;
    default: return -1;
  }
}
PathScope::PathScope(int path, std::atomic<int>* last) : prev_path(tl_path), prev_last(tl_last) {
  tl_path = path;
  tl_last = last;
}
PathScope::~PathScope() {
  tl_path = prev_path;
  tl_last = prev_last;
}
static std::atomic<int> g_last_path{0};
void note_path(int path) {
  g_last_path.store(path, std::memory_order_relaxed);
  if (tl_last) tl_last->store(path, std::memory_order_relaxed);
}
int last_path() { return g_last_path.load(std::memory_order_relaxed); }

me_status fail(me_ctx* c, me_status s, const char* fmt, ...) {
  if (c) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(c->err, sizeof c->err, fmt, ap);
    va_end(ap);
  }
  return s;
}

me_status grow(me_ctx* c, void** p, size_t* cap, size_t need) {
  if (*cap >= need && *p) return ME_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, need) != hipSuccess) {
    *p = nullptr;
    return fail(c, ME_ENOMEM, "hipMalloc(%zu) failed", need);
  }
  *cap = need;
  return ME_OK;
}

me_status check_args(me_ctx* c, const void* ref, const void* cur, int width, int height,
                     int stride, int blk, int range, int cost, const void* mv) {
  if (!c) return ME_EINVAL;
  if (!ref || !cur || !mv) return fail(c, ME_EINVAL, "null plane or output pointer");
  if (width <= 0 || height <= 0) return fail(c, ME_EINVAL, "frame %dx%d", width, height);
  if (stride < width) return fail(c, ME_EINVAL, "stride %d < width %d", stride, width);
  if (blk < 1 || blk > ME_MAX_BLOCK) return fail(c, ME_EINVAL, "block_size %d", blk);
  if (range < 0 || range > ME_MAX_RANGE) return fail(c, ME_EINVAL, "search_range %d", range);
  if (cost != ME_COST_SSD && cost != ME_COST_SAD && cost != ME_COST_SSIM)
    return fail(c, ME_EINVAL, "cost %d", cost);
  // Buffer descriptors carry 32-bit byte ranges: planes stay below 2 GiB.
  if ((long long)stride * height >= (1LL << 31))
    return fail(c, ME_EUNSUPPORTED, "plane of %lld bytes (limit 2 GiB)",
                (long long)stride * height);
  return ME_OK;
}

SearchArgs make_args(const uint8_t* ref, int ref_row0, const uint8_t* cur, int cur_row0,
                         int width, int height, int stride, int blk, int range, int cost,
                         int r0, int r1, int16_t* mv, uint32_t* cst) {
  SearchArgs p;
  p.ref = ref;
  p.cur = cur;
  p.ref_row0 = ref_row0;
  p.cur_row0 = cur_row0;
  p.width = width;
  p.height = height;
  p.stride = stride;
  p.blk = blk;
  p.range = range;
  p.nbx = (width + blk - 1) / blk;
  p.block_row_begin = r0;
  p.block_row_end = r1;
  p.cost_kind = cost;
  p.mv = mv;
  p.cost = cst;
  // Bytes the kernels may read from each plane (the DMA descriptors' range):
  // the rows the stripe contract guarantees resident (include/me.h).
  const int ref_end = r1 * blk + range < height ? r1 * blk + range : height;
  const int cur_end = r1 * blk < height ? r1 * blk : height;
  const long ref_rows = ref_end - ref_row0, cur_rows = cur_end - cur_row0;
  p.ref_bytes = ref_rows > 0 ? (uint32_t)((ref_rows - 1) * (long)stride + width) : 0;
  p.cur_bytes = cur_rows > 0 ? (uint32_t)((cur_rows - 1) * (long)stride + width) : 0;
  p.sched = nullptr;
  p.scratch = nullptr;
  p.scratch_bytes = 0;
  p.mkeys = nullptr;
  p.mcnt = nullptr;
  p.merge_tiles = 0;
  return p;
}

me_status attach_scratch(me_ctx* c, Dev& d, SearchArgs& p, bool cap, int batch) {
  ME_CTX_PATH_SCOPE(c, d);  // the scratch follows the kernels the context's path plans
  p.sched = d.sched;
  {
    const size_t tiles = merge_tiles_needed(p);
    if (tiles > d.merge_cap) {
      if (cap) return fail(c, ME_EINVAL, "captured search needs new scratch: run it once uncaptured first");
      (void)hipFree(d.mkeys);
      (void)hipFree(d.mcnt);
      d.mkeys = nullptr;
      d.mcnt = nullptr;
      d.merge_cap = 0;
      if (hipMalloc((void**)&d.mkeys, tiles * 16 * 8) != hipSuccess ||
          hipMalloc((void**)&d.mcnt, tiles * 4) != hipSuccess ||
          hipMemset(d.mkeys, 0xFF, tiles * 16 * 8) != hipSuccess ||
          hipMemset(d.mcnt, 0, tiles * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return fail(c, ME_ENOMEM, "MFMA merge buffers (%zu tiles)", tiles);
      d.merge_cap = tiles;
    }
  }
  p.mkeys = d.mkeys;
  p.mcnt = d.mcnt;
  p.merge_tiles = d.merge_cap;
  // a batch of equal jobs: prepass planes for a launch's worth of them
  size_t need = batch > 1 ? mfma_batch_scratch(p, batch) : mfma_ssd_scratch(p);
  const size_t ssim = ssim_scratch(p);  // SSIM jobs run one by one on one plane
  if (ssim > need) need = ssim;
  if (need && cap && (need > d.scratch_cap || !d.scratch))
    return fail(c, ME_EINVAL, "captured search needs new scratch: run it once uncaptured first");
  if (need) {
    me_status s = grow(c, (void**)&d.scratch, &d.scratch_cap, need);
    if (s != ME_OK) return s;
  }
  p.scratch = d.scratch;
  p.scratch_bytes = d.scratch ? d.scratch_cap : 0;
  return ME_OK;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return s && hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}

me_status order_on(me_ctx* c, Dev& d, hipStream_t s) {
  if (d.searched && d.search_stream != s) {
    // The event is recorded now, on the previous search's stream: it covers
    // that search (and whatever the caller queued after it there, which only
    // over-orders).  An event per search instead cost ~3 us of GPU time
    // between back-to-back searches (1080p 82.3 -> 79.3 us without it), and the
    // round-2 device-wide synchronisation at the first switch blocked the host
    // and drained unrelated streams.  The previous stream must still exist
    // (include/me.h: a stream stays valid until the next search is enqueued).
    HIPCHK(c, hipEventRecord(d.search_ev, d.search_stream));
    HIPCHK(c, hipStreamWaitEvent(s, d.search_ev, 0));
  }
  d.search_stream = s;
  d.searched = true;
  return ME_OK;
}

me_status launch_ordered(me_ctx* c, Dev& d, SearchArgs& p, hipStream_t s) {
  ME_CTX_PATH_SCOPE(c, d);
  // Captured launches run only when their graph does (me_graph_launch orders
  // it): no ordering and no state change at capture time.
  const bool cap = capturing(s);
  if (!cap) {
    me_status st = order_on(c, d, s);
    if (st != ME_OK) return st;
  }
  const hipError_t e = launch_search(p, s, nullptr);
  if (e != hipSuccess) {
    if (!cap) {
      (void)hipMemsetAsync(d.sched, 0, SCHED_WORDS * 4, s);
      if (d.mkeys) (void)hipMemsetAsync(d.mkeys, 0xFF, d.merge_cap * 16 * 8, s);
      if (d.mcnt) (void)hipMemsetAsync(d.mcnt, 0, d.merge_cap * 4, s);
    }
    return fail(c, ME_EDEVICE, "search launch: %s", hipGetErrorString(e));
  }
  return ME_OK;
}

me_status launch_jobs_ordered(me_ctx* c, Dev& d, const SearchArgs& base, const SearchJob* jobs,
                              int n, hipStream_t s, bool cap) {
  ME_CTX_PATH_SCOPE(c, d);
  if (!cap) {
    me_status st = order_on(c, d, s);
    if (st != ME_OK) return st;
  }
  const hipError_t e = launch_jobs(base, jobs, n, s);
  if (e != hipSuccess) {
    if (!cap) {
      (void)hipMemsetAsync(d.sched, 0, SCHED_WORDS * 4, s);
      if (d.mkeys) (void)hipMemsetAsync(d.mkeys, 0xFF, d.merge_cap * 16 * 8, s);
      if (d.mcnt) (void)hipMemsetAsync(d.mcnt, 0, d.merge_cap * 4, s);
    }
    return fail(c, ME_EDEVICE, "search launch: %s", hipGetErrorString(e));
  }
  return ME_OK;
}

me_status own_stream(me_ctx* c, Dev& d) {
  if (!d.stream) HIPCHK(c, hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  return ME_OK;
}

me_status device_status(me_ctx* c, Dev& d, hipStream_t s) {
  uint32_t w = 0;
  HIPCHK(c, hipMemcpyAsync(&w, d.sched + SCHED_ERR, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  if (w) {
    // The word is per device, so it may also hold the report of an earlier
    // asynchronous search that nobody checked yet: keep it for that caller's
    // me_device_check as well (include/me.h) -- when there is such a search.
    if (d.async_unchecked) d.err_pending = w;
    HIPCHK(c, hipMemsetAsync(d.sched + SCHED_ERR, 0, 4, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return fail(c, ME_EDEVICE, "device %d: a search kernel's bounded wait expired (code %u): "
                "the MV field of this or an earlier unchecked search on the device is invalid",
                d.id, w);
  }
  return ME_OK;
}

// ------------------------------------------------------------ host workers
Workers::Workers(int n) {
  th_.reserve(n);
  for (int i = 0; i < n; i++) th_.emplace_back(&Workers::loop, this, i);
}

Workers::~Workers() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  go_.notify_all();
  for (auto& t : th_) t.join();
}

void Workers::loop(int i) {
  unsigned long long seen = 0;
  for (;;) {
    const std::function<void(int)>* fn;
    int n, off;
    {
      std::unique_lock<std::mutex> lk(mu_);
      go_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      fn = fn_;
      n = n_;
      off = off_;
    }
    if (i < n) (*fn)(i + off);
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
}

void Workers::run(int n, const std::function<void(int)>& fn) {
  std::unique_lock<std::mutex> lk(mu_);
  fn_ = &fn;
  n_ = n;
  off_ = 0;
  pending_ = (int)th_.size();
  gen_++;
  go_.notify_all();
  done_.wait(lk, [&] { return pending_ == 0; });
  fn_ = nullptr;
}

void Workers::run_split(int n, const std::function<void(int)>& fn) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    fn_ = &fn;
    n_ = n - 1;
    off_ = 1;
    pending_ = (int)th_.size();
    gen_++;
  }
  go_.notify_all();
  fn(0);
  std::unique_lock<std::mutex> lk(mu_);
  done_.wait(lk, [&] { return pending_ == 0; });
  fn_ = nullptr;
}

Workers* workers(me_ctx* c) {
  if (!c->pool) {
    try {
      c->pool = new Workers((int)c->devs.size());
    } catch (...) {  // std::system_error: no thread could be started
      c->pool = nullptr;
    }
  }
  return c->pool;
}

// ------------------------------------------------- RCCL failure detection
me_status wait_comm(me_ctx* c, hipStream_t s, hipEvent_t ev, ncclComm_t comm, int timeout_ms) {
  HIPCHK(c, hipEventRecord(ev, s));
  const auto t0 = std::chrono::steady_clock::now();
  for (int spins = 0;; spins++) {
    const hipError_t q = hipEventQuery(ev);
    ncclResult_t ar = ncclSuccess;
    if (comm && ncclCommGetAsyncError(comm, &ar) == ncclSuccess && ar != ncclSuccess &&
        ar != ncclInProgress)
      return fail(c, ME_ECOMM, "RCCL reported an asynchronous error: %s (%s)",
                  ncclGetErrorString(ar), comm ? ncclGetLastError(comm) : "");
    if (q == hipSuccess) return ME_OK;
    if (q != hipErrorNotReady) return fail(c, ME_EDEVICE, "stream query: %s", hipGetErrorString(q));
    const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    if (ms >= timeout_ms)
      return fail(c, ME_ECOMM, "the collective did not complete within %d ms (a rank stalled "
                  "or died); the communicator is aborted", timeout_ms);
    // spin for the first ~0.1 ms (the usual case: the gather is microseconds
    // from done), then poll every 50 us
    if (spins < 200)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

}  // namespace me

namespace {

using me::fail;
using me::grow;
using me::check_args;
using me::make_args;
using me::attach_scratch;
using me::launch_ordered;

me_status ensure_comms(me_ctx* c) {
  if (c->comms || !c->distinct || c->devs.size() < 2) return ME_OK;
  const int n = (int)c->devs.size();
  std::vector<int> ids(n);
  for (int i = 0; i < n; i++) ids[i] = c->devs[i].id;
  c->comms = new (std::nothrow) ncclComm_t[n];
  if (!c->comms) return fail(c, ME_ENOMEM, "comm array");
  ncclResult_t r = ncclCommInitAll(c->comms, n, ids.data());
  if (r != ncclSuccess) {
    delete[] c->comms;
    c->comms = nullptr;
    return fail(c, ME_ECOMM, "ncclCommInitAll: %s", ncclGetErrorString(r));
  }
  return ME_OK;
}

// One stripe of a multi-device search on its device: upload the cur stripe
// and the ref rows with the S-row halo, then launch (the calling thread owns d).
me_status stripe_upload_launch(me_ctx* c, Dev& d, const uint8_t* ref, const uint8_t* cur,
                               int width, int height, int stride, int blk, int range, int cost,
                               int r0, int r1, size_t max_blocks) {
  HIPCHK(c, hipSetDevice(d.id));
  me_status s0 = me::own_stream(c, d);
  if (s0 != ME_OK) return s0;
  const int y_ref0 = r0 * blk - range > 0 ? r0 * blk - range : 0;
  const int y_ref1 = r1 * blk + range < height ? r1 * blk + range : height;
  const int y_cur0 = r0 * blk;
  const int y_cur1 = r1 * blk < height ? r1 * blk : height;
  const size_t ref_rows = r1 > r0 ? (size_t)(y_ref1 - y_ref0) : 0;
  const size_t cur_rows = r1 > r0 ? (size_t)(y_cur1 - y_cur0) : 0;
  me_status s;
  if ((s = grow(c, (void**)&d.ref, &d.frame_cap, (ref_rows + cur_rows + 1) * width)) != ME_OK)
    return s;
  d.cur = d.ref + ref_rows * width;
  if ((s = grow(c, (void**)&d.rec, &d.rec_cap, max_blocks * 8)) != ME_OK) return s;
  if (r1 <= r0) return ME_OK;
  HIPCHK(c, hipMemcpy2DAsync(d.ref, width, ref + (size_t)y_ref0 * stride, stride, width,
                             ref_rows, hipMemcpyHostToDevice, d.stream));
  HIPCHK(c, hipMemcpy2DAsync(d.cur, width, cur + (size_t)y_cur0 * stride, stride, width,
                             cur_rows, hipMemcpyHostToDevice, d.stream));
  int16_t* dmv = reinterpret_cast<int16_t*>(d.rec);
  uint32_t* dcost = reinterpret_cast<uint32_t*>(d.rec + max_blocks * 4);
  me::SearchArgs p = make_args(d.ref, y_ref0, d.cur, y_cur0, width, height, width, blk, range,
                               cost, r0, r1, dmv, dcost);
  if ((s = attach_scratch(c, d, p)) != ME_OK) return s;
  return launch_ordered(c, d, p, d.stream);
}

// Multi-device frame search: row stripes balanced by me_plan_stripes' per-row
// cost model (include/me.h), one per context device.  One host thread per device uploads its stripe
// (pageable host planes are staged by the runtime, so the uploads of the
// devices overlap instead of running one after another) and enqueues its
// search; then one ncclGather of the padded per-stripe records to device 0.
me_status multi_search(me_ctx* c, const uint8_t* ref, const uint8_t* cur, int width,
                       int height, int stride, int blk, int range, int cost, int16_t* mv_xy,
                       uint32_t* block_cost) {
  const int n = (int)c->devs.size();
  const int nbx = (width + blk - 1) / blk;
  std::vector<int> bounds(n + 1);
  me_status s = me_plan_stripes(width, height, blk, range, n, bounds.data());
  if (s != ME_OK) return fail(c, s, "stripe plan");
  int max_rows = 0;
  for (int i = 0; i < n; i++)
    max_rows = bounds[i + 1] - bounds[i] > max_rows ? bounds[i + 1] - bounds[i] : max_rows;
  const size_t max_blocks = (size_t)(max_rows > 0 ? max_rows : 1) * nbx;
  const size_t rec_bytes = max_blocks * 8;

  {
    // one persistent host thread per device (me::Workers), not threads per call
    me::Workers* pool = me::workers(c);
    if (!pool) return fail(c, ME_ENOMEM, "host worker threads");
    std::vector<me_ctx> errs(n);
    for (me_ctx& e : errs) e.owner = c;
    std::vector<me_status> st(n, ME_OK);
    pool->run(n, [&](int i) {
      st[i] = stripe_upload_launch(&errs[i], c->devs[i], ref, cur, width, height, stride, blk,
                                   range, cost, bounds[i], bounds[i + 1], max_blocks);
    });
    for (int i = 0; i < n; i++)
      if (st[i] != ME_OK) return fail(c, st[i], "device %d: %s", c->devs[i].id, errs[i].err);
  }
  Dev& root = c->devs[0];
  HIPCHK(c, hipSetDevice(root.id));
  if ((s = grow(c, (void**)&root.gather, &root.gather_cap, rec_bytes * n)) != ME_OK) return s;
  if (c->distinct) {
    if ((s = ensure_comms(c)) != ME_OK) return s;
    // The searches end on their own (their kernels' waits are bounded): mark
    // each one's end, so that the bounded RCCL wait below covers the gather
    // alone, not a long search (8K 8x8 SSIM at a large range takes minutes).
    std::vector<hipEvent_t> done(n, nullptr);
    auto drop = [&]() {
      for (int i = 0; i < n; i++)
        if (done[i]) (void)hipEventDestroy(done[i]);
    };
    for (int i = 0; i < n; i++) {
      Dev& d = c->devs[i];
      if (hipSetDevice(d.id) != hipSuccess ||
          hipEventCreateWithFlags(&done[i], hipEventDisableTiming) != hipSuccess ||
          hipEventRecord(done[i], d.stream) != hipSuccess) {
        drop();
        return fail(c, ME_EDEVICE, "device %d: search end event", d.id);
      }
    }
    HIPCHK(c, hipSetDevice(root.id));
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < n && r == ncclSuccess; i++) {
      Dev& d = c->devs[i];
      r = ncclGather(d.rec, i == 0 ? root.gather : nullptr, rec_bytes, ncclUint8, 0, c->comms[i],
                     d.stream);
    }
    const ncclResult_t re = ncclGroupEnd();
    if (r == ncclSuccess) r = re;
    if (r != ncclSuccess) {
      drop();
      return fail(c, ME_ECOMM, "ncclGather: %s", ncclGetErrorString(r));
    }
    // Bounded wait on every device's gather, started once its search is done:
    // a device that stalls (or an RCCL error) aborts the group instead of
    // blocking this call forever; the next search builds a new one.
    for (int i = 0; i < n; i++) {
      Dev& d = c->devs[i];
      HIPCHK(c, hipSetDevice(d.id));
      const hipError_t e = hipEventSynchronize(done[i]);
      s = e == hipSuccess ? me::wait_comm(c, d.stream, d.search_ev, c->comms[i], ME_COMM_TIMEOUT_MS)
                          : fail(c, ME_EDEVICE, "device %d search: %s", d.id, hipGetErrorString(e));
      if (s != ME_OK) {
        for (int k = 0; k < n; k++) (void)ncclCommAbort(c->comms[k]);
        delete[] c->comms;
        c->comms = nullptr;
        drop();
        return s;
      }
    }
    drop();
  } else {
    // Repeated device ids: stripes share a device; device copies stand in for the gather.
    for (int i = 0; i < n; i++) {
      Dev& d = c->devs[i];
      HIPCHK(c, hipStreamSynchronize(d.stream));
      HIPCHK(c, hipMemcpyPeerAsync(root.gather + i * rec_bytes, root.id, d.rec, d.id, rec_bytes,
                                   root.stream));
    }
  }
  for (int i = 0; i < n; i++) {
    HIPCHK(c, hipSetDevice(c->devs[i].id));
    if ((s = me::device_status(c, c->devs[i], c->devs[i].stream)) != ME_OK) return s;
  }
  HIPCHK(c, hipSetDevice(root.id));
  std::vector<uint8_t> host(rec_bytes * n);
  HIPCHK(c, hipMemcpy(host.data(), root.gather, host.size(), hipMemcpyDeviceToHost));
  for (int i = 0; i < n; i++) {
    const int nblk = (bounds[i + 1] - bounds[i]) * nbx;
    const uint8_t* base = host.data() + i * rec_bytes;
    const size_t off = (size_t)bounds[i] * nbx;
    memcpy(mv_xy + 2 * off, base, (size_t)nblk * 4);
    if (block_cost) memcpy(block_cost + off, base + max_blocks * 4, (size_t)nblk * 4);
  }
  return ME_OK;
}

}  // namespace

extern "C" {

const char* me_status_str(me_status s) {
  switch (s) {
    case ME_OK: return "ok";
    case ME_EINVAL: return "invalid argument";
    case ME_ENOMEM: return "out of memory";
    case ME_EDEVICE: return "device error";
    case ME_ECOMM: return "communication error";
    case ME_EUNSUPPORTED: return "unsupported";
    case ME_EIO: return "i/o error";
  }
  return "unknown status";
}

const char* me_last_error(const me_ctx* ctx) { return ctx ? ctx->err : "null context"; }

const char* me_version(void) { return "me_hip 1 gfx950"; }

int me_last_search_path(void) { return me::last_path(); }

void me_set_kernel_path(me_path path) {
  const int code = me::path_code_of((int)path);
  me::set_kernel_path_code(code < 0 ? 0 : code);
}

me_status me_ctx_set_kernel_path(me_ctx* c, int path) {
  if (!c) return ME_EINVAL;
  if (path == ME_PATH_PROCESS) {
    c->path = -1;
    return ME_OK;
  }
  const int code = me::path_code_of(path);
  if (code < 0) return me::fail(c, ME_EINVAL, "me_ctx_set_kernel_path: unknown path %d", path);
  c->path = code;
  return ME_OK;
}

int me_ctx_last_search_path(const me_ctx* c, int device_index) {
  if (!c || device_index < 0 || (size_t)device_index >= c->last_path.size()) return -1;
  return c->last_path[(size_t)device_index].load(std::memory_order_relaxed);
}

me_status me_create(me_ctx** out, const int* device_ids, int n) {
  if (!out) return ME_EINVAL;
  *out = nullptr;
  me_ctx* c = new (std::nothrow) me_ctx();
  if (!c) return ME_ENOMEM;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count < 1) {
    delete c;
    return ME_EDEVICE;
  }
  std::vector<int> ids;
  if (!device_ids || n <= 0) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) cur = 0;
    ids.push_back(cur);
  } else {
    for (int i = 0; i < n; i++) {
      if (device_ids[i] < 0 || device_ids[i] >= count) {
        delete c;
        return ME_EINVAL;
      }
      ids.push_back(device_ids[i]);
    }
  }
  for (size_t i = 0; i < ids.size(); i++)
    for (size_t j = 0; j < i; j++)
      if (ids[i] == ids[j]) c->distinct = false;
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (int id : ids) {
    Dev d;
    d.id = id;
    if (hipSetDevice(id) != hipSuccess ||
        hipMalloc((void**)&d.sched, me::SCHED_WORDS * 4) != hipSuccess ||
        hipMemset(d.sched, 0, me::SCHED_WORDS * 4) != hipSuccess ||
        hipEventCreateWithFlags(&d.search_ev, hipEventDisableTiming) != hipSuccess) {
      c->devs.push_back(d);
      me_destroy(c);
      (void)hipSetDevice(prev);
      return ME_EDEVICE;
    }
    c->devs.push_back(d);
  }
  (void)hipSetDevice(prev);
  c->last_path = std::vector<std::atomic<int>>(c->devs.size());
  for (auto& a : c->last_path) a.store(ME_SEARCH_PATH_NONE, std::memory_order_relaxed);
  *out = c;
  return ME_OK;
}

me_status me_comm_unique_id(void* id) {
  if (!id) return ME_EINVAL;
  static_assert(sizeof(ncclUniqueId) == ME_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return ME_ECOMM;
  memcpy(id, &u, sizeof(u));
  return ME_OK;
}

me_status me_comm_init(me_ctx* c, const void* id, int n_ranks, int rank) {
  if (!c) return ME_EINVAL;
  if (!id || n_ranks < 1 || rank < 0 || rank >= n_ranks)
    return fail(c, ME_EINVAL, "comm rank %d of %d", rank, n_ranks);
  if (c->rank_comm) return fail(c, ME_EINVAL, "communicator already initialised");
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  int prev = 0;
  (void)hipGetDevice(&prev);
  HIPCHK(c, hipSetDevice(c->devs[0].id));
  ncclComm_t comm = nullptr;
  const ncclResult_t r = ncclCommInitRank(&comm, n_ranks, u, rank);
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) return fail(c, ME_ECOMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
  c->rank_comm = comm;
  c->comm_ranks = n_ranks;
  c->comm_rank = rank;
  c->comm_aborted = false;  // a communicator rebuilt after me_comm_check aborted the last one
  return ME_OK;
}

me_status me_gather_device(me_ctx* c, const void* d_send, size_t bytes, void* d_recv,
                           void* stream) {
  if (!c) return ME_EINVAL;
  if (c->comm_aborted)
    return fail(c, ME_ECOMM, "the communicator was aborted by me_comm_check (a failed exchange)");
  if (!c->rank_comm) return fail(c, ME_EINVAL, "me_comm_init was not called");
  if (!d_send || (c->comm_rank == 0 && !d_recv)) return fail(c, ME_EINVAL, "null buffer");
  NCCLCHK(c, ncclGather(d_send, c->comm_rank == 0 ? d_recv : nullptr, bytes, ncclUint8, 0,
                        c->rank_comm, reinterpret_cast<hipStream_t>(stream)));
  return ME_OK;
}

me_status me_comm_check(me_ctx* c, void* stream, int timeout_ms) {
  if (!c) return ME_EINVAL;
  if (c->comm_aborted)
    return fail(c, ME_ECOMM, "the communicator was aborted by an earlier me_comm_check");
  if (!c->rank_comm) return fail(c, ME_EINVAL, "me_comm_init was not called");
  if (timeout_ms < 0) return fail(c, ME_EINVAL, "timeout_ms %d", timeout_ms);
  int prev = 0;
  (void)hipGetDevice(&prev);
  HIPCHK(c, hipSetDevice(c->devs[0].id));
  if (!c->comm_ev) HIPCHK(c, hipEventCreateWithFlags(&c->comm_ev, hipEventDisableTiming));
  me_status s = me::wait_comm(c, (hipStream_t)stream, c->comm_ev, c->rank_comm, timeout_ms);
  if (s == ME_ECOMM) {
    // Abort: RCCL's kernels on this rank return, so the stream (and every
    // stream synchronisation after it) can finish instead of hanging.
    (void)ncclCommAbort(c->rank_comm);
    c->rank_comm = nullptr;
    c->comm_aborted = true;
  }
  (void)hipSetDevice(prev);
  return s;
}

me_status me_device_check(me_ctx* c) {
  if (!c) return ME_EINVAL;
  int prev = 0;
  (void)hipGetDevice(&prev);
  me_status s = ME_OK;
  for (Dev& d : c->devs) {
    d.async_unchecked = false;
    uint32_t w = 0;
    if (hipSetDevice(d.id) != hipSuccess ||
        hipMemcpy(&w, d.sched + me::SCHED_ERR, 4, hipMemcpyDeviceToHost) != hipSuccess) {
      s = fail(c, ME_EDEVICE, "device %d: reading the invariant word failed", d.id);
      break;
    }
    if (w || d.err_pending) {
      if (w) (void)hipMemset(d.sched + me::SCHED_ERR, 0, 4);
      s = fail(c, ME_EDEVICE, "device %d: a search kernel's bounded wait expired (code %u%s): "
               "the MV field of that search is invalid", d.id, w ? w : d.err_pending,
               w ? "" : ", first reported to a synchronous call");
      d.err_pending = 0;
      break;
    }
  }
  (void)hipSetDevice(prev);
  return s;
}

// A captured step: the graph plus what its searches point into.
struct me_graph {
  me_ctx* ctx;
  hipGraphExec_t exec;
  const void *sched, *scratch, *mkeys, *mcnt;
};

me_status me_capture_begin(me_ctx* c, void* stream) {
  if (!c) return ME_EINVAL;
  if (!stream) return fail(c, ME_EINVAL, "capture needs a created stream, not the NULL stream");
  c->err[0] = 0;
  HIPCHK(c, hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeRelaxed));
  return ME_OK;
}

me_status me_capture_end(me_ctx* c, void* stream, me_graph** out) {
  if (!c) return ME_EINVAL;
  if (!out) return fail(c, ME_EINVAL, "null graph pointer");
  *out = nullptr;
  hipGraph_t g = nullptr;
  HIPCHK(c, hipStreamEndCapture((hipStream_t)stream, &g));
  hipGraphExec_t ex = nullptr;
  const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  HIPCHK(c, e);
  const Dev& d = c->devs[0];
  me_graph* gr = new (std::nothrow) me_graph{c, ex, d.sched, d.scratch, d.mkeys, d.mcnt};
  if (!gr) {
    (void)hipGraphExecDestroy(ex);
    return fail(c, ME_ENOMEM, "graph");
  }
  *out = gr;
  return ME_OK;
}

me_status me_graph_launch(me_graph* g, void* stream) {
  if (!g) return ME_EINVAL;
  me_ctx* c = g->ctx;
  Dev& d = c->devs[0];
  if (d.sched != g->sched || d.scratch != g->scratch || d.mkeys != g->mkeys || d.mcnt != g->mcnt)
    return fail(c, ME_EINVAL, "the context's search scratch was regrown after capture: capture again");
  me_status s = me::order_on(c, d, (hipStream_t)stream);
  if (s != ME_OK) return s;
  HIPCHK(c, hipGraphLaunch(g->exec, (hipStream_t)stream));
  d.async_unchecked = true;
  return ME_OK;
}

void me_graph_destroy(me_graph* g) {
  if (!g) return;
  (void)hipGraphExecDestroy(g->exec);
  delete g;
}

void me_destroy(me_ctx* c) {
  if (!c) return;
  delete c->pool;  // joins the idle workers
  c->pool = nullptr;
  if (c->rank_comm) ncclCommDestroy(c->rank_comm);
  if (c->comm_ev) (void)hipEventDestroy(c->comm_ev);
  if (c->comms) {
    for (size_t i = 0; i < c->devs.size(); i++) ncclCommDestroy(c->comms[i]);
    delete[] c->comms;
  }
  for (Dev& d : c->devs) {
    (void)hipSetDevice(d.id);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    (void)hipFree(d.ref);
    (void)hipFree(d.rec);
    (void)hipFree(d.gather);
    (void)hipFree(d.stats);
    (void)hipFree(d.out5);
    (void)hipFree(d.sched);
    (void)hipFree(d.scratch);
    (void)hipFree(d.mkeys);
    (void)hipFree(d.mcnt);
    me::release_pipeline(d);
    if (d.search_ev) (void)hipEventDestroy(d.search_ev);
    if (d.stream) (void)hipStreamDestroy(d.stream);
  }
  delete c;
}

me_status me_full_search(me_ctx* c, const uint8_t* ref, const uint8_t* cur, int width,
                         int height, int stride, int blk, int range, me_cost cost,
                         int16_t* mv_xy, uint32_t* block_cost) {
  me_status s = check_args(c, ref, cur, width, height, stride, blk, range, cost, mv_xy);
  if (s != ME_OK) return s;
  c->err[0] = 0;
  if (c->devs.size() > 1)
    return multi_search(c, ref, cur, width, height, stride, blk, range, cost, mv_xy, block_cost);
  Dev& d = c->devs[0];
  HIPCHK(c, hipSetDevice(d.id));
  if ((s = me::own_stream(c, d)) != ME_OK) return s;
  const size_t plane = (size_t)width * height;
  const size_t nb = (size_t)me_num_blocks(width, height, blk);
  if ((s = grow(c, (void**)&d.ref, &d.frame_cap, 2 * plane)) != ME_OK) return s;
  d.cur = d.ref + plane;
  if ((s = grow(c, (void**)&d.rec, &d.rec_cap, nb * 8)) != ME_OK) return s;
  HIPCHK(c, hipMemcpy2DAsync(d.ref, width, ref, stride, width, height, hipMemcpyHostToDevice, d.stream));
  HIPCHK(c, hipMemcpy2DAsync(d.cur, width, cur, stride, width, height, hipMemcpyHostToDevice, d.stream));
  int16_t* dmv = reinterpret_cast<int16_t*>(d.rec);
  uint32_t* dcost = reinterpret_cast<uint32_t*>(d.rec + nb * 4);
  const int nby = (height + blk - 1) / blk;
  me::SearchArgs p = make_args(d.ref, 0, d.cur, 0, width, height, width, blk, range, cost, 0,
                               nby, dmv, dcost);
  if ((s = attach_scratch(c, d, p)) != ME_OK) return s;
  if ((s = launch_ordered(c, d, p, d.stream)) != ME_OK) return s;
  HIPCHK(c, hipMemcpyAsync(mv_xy, dmv, nb * 4, hipMemcpyDeviceToHost, d.stream));
  if (block_cost)
    HIPCHK(c, hipMemcpyAsync(block_cost, dcost, nb * 4, hipMemcpyDeviceToHost, d.stream));
  return me::device_status(c, d, d.stream);
}

me_status me_full_search_stripe_device(me_ctx* c, const uint8_t* d_ref, int ref_row0,
                                       const uint8_t* d_cur, int cur_row0, int width,
                                       int height, int stride, int blk, int range, me_cost cost,
                                       int r0, int r1, int16_t* d_mv, uint32_t* d_cost,
                                       void* stream) {
  me_status s = check_args(c, d_ref, d_cur, width, height, stride, blk, range, cost, d_mv);
  if (s != ME_OK) return s;
  const int nby = (height + blk - 1) / blk;
  if (r0 < 0 || r1 > nby || r0 > r1) return fail(c, ME_EINVAL, "block rows [%d, %d)", r0, r1);
  const int need_ref0 = r0 * blk - range > 0 ? r0 * blk - range : 0;
  if (ref_row0 < 0 || ref_row0 > need_ref0) return fail(c, ME_EINVAL, "ref_row0 %d", ref_row0);
  if (cur_row0 < 0 || cur_row0 > r0 * blk) return fail(c, ME_EINVAL, "cur_row0 %d", cur_row0);
  c->err[0] = 0;
  me::SearchArgs p = make_args(d_ref, ref_row0, d_cur, cur_row0, width, height, stride, blk,
                               range, cost, r0, r1, d_mv, d_cost);
  const bool cap = me::capturing((hipStream_t)stream);
  if ((s = attach_scratch(c, c->devs[0], p, cap)) != ME_OK) return s;
  if ((s = launch_ordered(c, c->devs[0], p, (hipStream_t)stream)) != ME_OK) return s;
  c->devs[0].async_unchecked = true;
  return ME_OK;
}

me_status me_search_stripes_device(me_ctx* c, int width, int height, int stride, int blk,
                                   int range, me_cost cost, const me_stripe_job* jobs, int n_jobs,
                                   void* stream) {
  if (!c) return ME_EINVAL;
  if (!jobs || n_jobs < 0) return fail(c, ME_EINVAL, "job list");
  if (n_jobs == 0) return ME_OK;
  const int nby = blk > 0 ? (height + blk - 1) / blk : 0;
  std::vector<me::SearchJob> js((size_t)n_jobs);
  me::SearchArgs base{};
  Dev& d = c->devs[0];
  const bool cap = me::capturing((hipStream_t)stream);
  for (int i = 0; i < n_jobs; i++) {
    const me_stripe_job& J = jobs[i];
    me_status s = check_args(c, J.d_ref, J.d_cur, width, height, stride, blk, range, cost,
                             J.d_mv_xy);
    if (s != ME_OK) return s;
    const int r0 = J.block_row_begin, r1 = J.block_row_end;
    if (r0 < 0 || r1 > nby || r0 > r1)
      return fail(c, ME_EINVAL, "job %d: block rows [%d, %d)", i, r0, r1);
    const int need_ref0 = r0 * blk - range > 0 ? r0 * blk - range : 0;
    if (J.ref_row0 < 0 || J.ref_row0 > need_ref0)
      return fail(c, ME_EINVAL, "job %d: ref_row0 %d", i, J.ref_row0);
    if (J.cur_row0 < 0 || J.cur_row0 > r0 * blk)
      return fail(c, ME_EINVAL, "job %d: cur_row0 %d", i, J.cur_row0);
    js[i] = me::SearchJob{J.d_ref, J.ref_row0, J.d_cur, J.cur_row0, r0, r1, J.d_mv_xy, J.d_block_cost};
    // grow the device scratch to the largest job (the MFMA SSD path runs job by job)
    me::SearchArgs p = make_args(J.d_ref, J.ref_row0, J.d_cur, J.cur_row0, width, height, stride,
                                 blk, range, cost, r0, r1, J.d_mv_xy, J.d_block_cost);
    if ((s = attach_scratch(c, d, p, cap)) != ME_OK) return s;
  }
  // geometry, cost and the (final) scratch buffers every job's launch takes
  base = make_args(jobs[0].d_ref, jobs[0].ref_row0, jobs[0].d_cur, jobs[0].cur_row0, width, height,
                   stride, blk, range, cost, jobs[0].block_row_begin, jobs[0].block_row_end,
                   jobs[0].d_mv_xy, jobs[0].d_block_cost);
  {
    // jobs of one geometry (a batch of whole frames) share the SSD launches
    bool same = true;
    for (int i = 1; i < n_jobs; i++)
      same = same && jobs[i].block_row_begin == jobs[0].block_row_begin &&
             jobs[i].block_row_end == jobs[0].block_row_end && jobs[i].ref_row0 == jobs[0].ref_row0 &&
             jobs[i].cur_row0 == jobs[0].cur_row0;
    me_status s = attach_scratch(c, d, base, cap, same ? n_jobs : 1);
    if (s != ME_OK) return s;
  }
  c->err[0] = 0;
  me_status s = me::launch_jobs_ordered(c, d, base, js.data(), n_jobs, (hipStream_t)stream, cap);
  if (s == ME_OK) d.async_unchecked = true;
  return s;
}

me_status me_full_search_batch_device(me_ctx* c, const uint8_t* d_ref, size_t ref_frame_stride,
                                     int ref_row0, const uint8_t* d_cur, size_t cur_frame_stride,
                                     int cur_row0, int width, int height, int stride, int blk,
                                     int range, me_cost cost, int r0, int r1, int n_frames,
                                     int16_t* d_mv, uint32_t* d_cost, void* stream) {
  if (!c) return ME_EINVAL;
  if (n_frames < 1 || n_frames > 4096) return fail(c, ME_EINVAL, "n_frames %d", n_frames);
  me_status s = check_args(c, d_ref, d_cur, width, height, stride, blk, range, cost, d_mv);
  if (s != ME_OK) return s;
  const int nby = (height + blk - 1) / blk;
  if (r0 < 0 || r1 > nby || r0 > r1) return fail(c, ME_EINVAL, "block rows [%d, %d)", r0, r1);
  // every frame's resident rows inside its stride (frames must not overlap)
  const me::SearchArgs p = make_args(d_ref, ref_row0, d_cur, cur_row0, width, height, stride, blk,
                                     range, cost, r0, r1, d_mv, d_cost);
  if (n_frames > 1 && (ref_frame_stride < p.ref_bytes || cur_frame_stride < p.cur_bytes))
    return fail(c, ME_EINVAL, "frame strides %zu / %zu below a frame's %u / %u bytes",
                ref_frame_stride, cur_frame_stride, p.ref_bytes, p.cur_bytes);
  // One plane stack per batch, below 2 GiB like a single plane (check_args):
  // a stride past it is a caller error, refused before any frame address is
  // formed (a wild stride would otherwise send the kernels to unmapped memory).
  const unsigned long long rb = (unsigned long long)(n_frames - 1) * ref_frame_stride + p.ref_bytes;
  const unsigned long long cb = (unsigned long long)(n_frames - 1) * cur_frame_stride + p.cur_bytes;
  if (rb >= (1ull << 31) || cb >= (1ull << 31))
    return fail(c, ME_EUNSUPPORTED, "batch of %llu / %llu bytes (limit 2 GiB)", rb, cb);
  const size_t nblk = (size_t)(r1 - r0) * ((width + blk - 1) / blk);
  std::vector<me_stripe_job> jobs((size_t)n_frames);
  for (int f = 0; f < n_frames; f++)
    jobs[f] = me_stripe_job{d_ref + (size_t)f * ref_frame_stride, ref_row0,
                            d_cur + (size_t)f * cur_frame_stride, cur_row0, r0, r1,
                            d_mv + 2 * (size_t)f * nblk, d_cost ? d_cost + (size_t)f * nblk : nullptr};
  return me_search_stripes_device(c, width, height, stride, blk, range, cost, jobs.data(),
                                  n_frames, stream);
}

me_status me_full_search_device(me_ctx* c, const uint8_t* d_ref, const uint8_t* d_cur,
                                int width, int height, int stride, int blk, int range,
                                me_cost cost, int16_t* d_mv, uint32_t* d_cost, void* stream) {
  const int nby = blk > 0 ? (height + blk - 1) / blk : 0;
  return me_full_search_stripe_device(c, d_ref, 0, d_cur, 0, width, height, stride, blk, range,
                                      cost, 0, nby, d_mv, d_cost, stream);
}

me_status me_find_best_blocks(me_ctx* c, const int* ref_frame, const int* cur_frame, int width,
                              int height, int blk, int range, me_ref_block* blks, int num_blks) {
  me_status s = check_args(c, ref_frame, cur_frame, width, height, width, blk, range,
                           ME_COST_SSD, blks);
  if (s != ME_OK) return s;
  const int nb = me_num_blocks(width, height, blk);
  if (num_blks != nb) return fail(c, ME_EINVAL, "num_blks %d != %d", num_blks, nb);
  const size_t plane = (size_t)width * height;
  std::vector<uint8_t> r8(plane), c8(plane);
  for (size_t i = 0; i < plane; i++) {  // utils.c:49-53 widened u8 -> int; narrow back
    const int rv = ref_frame[i], cv = cur_frame[i];
    // the planes came from 8-bit files: anything else would be searched as
    // its low byte and give a field the reference would not
    if ((unsigned)rv > 255u || (unsigned)cv > 255u)
      return fail(c, ME_EINVAL, "pixel %zu (%d, %d) outside [0, 255]", i, rv, cv);
    r8[i] = (uint8_t)rv;
    c8[i] = (uint8_t)cv;
  }
  std::vector<int16_t> mv((size_t)nb * 2);
  s = me_full_search(c, r8.data(), c8.data(), width, height, width, blk, range, ME_COST_SSD,
                     mv.data(), nullptr);
  if (s != ME_OK) return s;
  for (int i = 0; i < nb; i++) {  // populateBlkMotionVector, main.c:11-15
    blks[i].motion_vectorX = mv[2 * i];
    blks[i].motion_vectorY = mv[2 * i + 1];
    blks[i].is_best_match_found = 1;
  }
  return ME_OK;
}

static me_status compensate(me_ctx* c, const uint8_t* ref, const uint8_t* cur, int width,
                            int height, int blk, const int16_t* mv_xy, uint8_t* out,
                            int planes, double* psnr) {
  me_status s = check_args(c, ref, cur ? cur : ref, width, height, width, blk, 0, ME_COST_SSD, mv_xy);
  if (s != ME_OK) return s;
  if (!out) return fail(c, ME_EINVAL, "null output");
  Dev& d = c->devs[0];
  HIPCHK(c, hipSetDevice(d.id));
  if ((s = me::own_stream(c, d)) != ME_OK) return s;
  const size_t plane = (size_t)width * height;
  const size_t nb = (size_t)me_num_blocks(width, height, blk);
  if ((s = grow(c, (void**)&d.ref, &d.frame_cap, 2 * plane)) != ME_OK) return s;
  d.cur = d.ref + plane;
  if ((s = grow(c, (void**)&d.rec, &d.rec_cap, nb * 8)) != ME_OK) return s;
  size_t scap = d.stats ? 16 : 0;
  if ((s = grow(c, (void**)&d.stats, &scap, 16)) != ME_OK) return s;
  const size_t out_bytes = planes ? 5 * plane : plane;
  if ((s = grow(c, (void**)&d.out5, &d.out_cap, out_bytes)) != ME_OK) return s;
  HIPCHK(c, hipMemcpyAsync(d.ref, ref, plane, hipMemcpyHostToDevice, d.stream));
  HIPCHK(c, hipMemcpyAsync(d.cur, cur ? cur : ref, plane, hipMemcpyHostToDevice, d.stream));
  HIPCHK(c, hipMemcpyAsync(d.rec, mv_xy, nb * 4, hipMemcpyHostToDevice, d.stream));
  HIPCHK(c, hipMemsetAsync(d.stats, 0, 16, d.stream));
  HIPCHK(c, me::launch_compensate(d.ref, d.cur, width, height, blk,
                                  reinterpret_cast<int16_t*>(d.rec), d.out5, planes, d.stats,
                                  d.stream));
  unsigned long long st[2] = {0, 0};
  HIPCHK(c, hipMemcpyAsync(out, d.out5, out_bytes, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(c, hipMemcpyAsync(st, d.stats, 16, hipMemcpyDeviceToHost, d.stream));
  HIPCHK(c, hipStreamSynchronize(d.stream));
  if (psnr) {  // utils.c:147-154, double arithmetic on the exact integer sum
    double mse = (double)st[0];
    mse /= (double)width * height;
    *psnr = mse == 0 ? 99.0 : 20 * log10((double)st[1]) - 10 * log10(mse);
  }
  return ME_OK;
}

me_status me_motion_compensate(me_ctx* c, const uint8_t* ref, int width, int height, int blk,
                               const int16_t* mv_xy, uint8_t* mc) {
  return compensate(c, ref, nullptr, width, height, blk, mv_xy, mc, 0, nullptr);
}

me_status me_compensate_planes(me_ctx* c, const uint8_t* ref, const uint8_t* cur, int width,
                               int height, int blk, const int16_t* mv_xy, uint8_t* out5,
                               double* psnr) {
  if (!cur) return fail(c, ME_EINVAL, "null cur");
  return compensate(c, ref, cur, width, height, blk, mv_xy, out5, 1, psnr);
}

}  // extern "C"
