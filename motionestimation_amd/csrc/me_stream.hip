// me_stream.hip -- frame-pair streaming and pinned host memory.
//
// The reference searches one (ref, cur) pair per process (src/cpu/main.c:109-179:
// read two frames, search, write, exit).  me_search_pairs takes a list of
// frames and a list of (ref, cur) index pairs -- consecutive pairs of a
// sequence, or one reference against several currents (the 1->2 and 1->4
// pairs of frames/ForemanYF{1,2,4}) -- and keeps every device busy:
//   - each frame is uploaded once per device, into a device slot that lives
//     from the first to the last pair reading it;
//   - pairs are searched in job-table launches (launch_jobs) ramping 1, 2, 3,
//     4, 6, 9 and then 12 pairs (pageable frames: 1, 2, 3, 4, 6, then 8): a
//     launch's fill and drain are paid once per batch, and the first search
//     starts after two uploads (profiles/r04h_*);
//   - pinned frames upload one batch ahead of the searches, and a batch's
//     frames that are adjacent in host memory and in their device slots go up
//     in one copy (round 6);
//   - uploads run on a copy stream, searches on the compute stream; the
//     host-side staging and upload of pair n+1's new frame overlap the search
//     of pair n (slots are reused oldest-freed first, so an upload never
//     waits on the search it should overlap);
//   - the streams are ordered by one event per batch each way (uploads done,
//     search done), not per frame slot: event packets between two search
//     launches delayed each launch by 58-74 us (profiles/r04e_*);
//   - frames in me_host_alloc memory are DMAed directly, other frames are
//     staged through two pinned buffers;
//   - each batch's MV records are downloaded (pinned bounce buffer, copy
//     stream) after its search and moved to the caller's arrays while later
//     batches search: one copy at the end took 250 us at 64 1080p pairs.
// With several context devices the pair list is cut into contiguous runs,
// one per device, each driven by its own host thread (independent pairs: no
// collective).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "me_internal.h"

namespace me {

namespace {
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pinned;  // me_host_alloc ranges: base -> bytes
// Freed frame slots kept cooling before reuse (ME_STREAM_COOL overrides; tuning)
static int cooling_slots() { return tuning().stream_cool > 0 ? tuning().stream_cool : 2; }
// Pairs per search launch after the ramp (ME_STREAM_BATCH overrides; tuning).
// With uploads one batch ahead and merged copies, pinned 1080p pairs/s over two
// sweeps: 8: 14.16k / 14.36k, 12: 14.42k / 14.50k, 16: 14.32k / 14.09k, 24:
// 13.94k / 14.37k, 32: 14.13k / 14.27k (profiles/r06x_stream_batch.jsonl;
// box noise ~2 %).  Round 5 (no lookahead): 8 was best.
constexpr int kPairBatch = 12;
constexpr int kEvRing = 16;  // batch events (Dev::upl_ev / batch_ev), ring by batch index
}  // namespace

bool host_range_pinned(const void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  const uintptr_t a = (uintptr_t)p;
  auto it = g_pinned.upper_bound(a);
  if (it == g_pinned.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->first + it->second;
}

void release_pipeline(Dev& d) {
  if (d.copy) (void)hipStreamSynchronize(d.copy);
  if (d.d2h) (void)hipStreamSynchronize(d.d2h);
  for (size_t i = 0; i < d.slot_chunks.size(); i++) (void)hipFree(d.slot_chunks[i]);
  d.slot_chunks.clear();
  d.slot_spare.clear();
  for (int k = 0; k < kEvRing; k++) {
    if (d.upl_ev[k]) (void)hipEventDestroy(d.upl_ev[k]);
    if (d.batch_ev[k]) (void)hipEventDestroy(d.batch_ev[k]);
    if (d.d2h_ev[k]) (void)hipEventDestroy(d.d2h_ev[k]);
    d.upl_ev[k] = d.batch_ev[k] = d.d2h_ev[k] = nullptr;
  }
  if (d.bounce) (void)hipHostFree(d.bounce);
  d.bounce = nullptr;
  d.bounce_cap = 0;
  if (d.d2h) (void)hipStreamDestroy(d.d2h);
  d.d2h = nullptr;
  d.slots.clear();
  d.slot_bytes = 0;
  for (int k = 0; k < 2; k++) {
    if (d.stage[k]) (void)hipHostFree(d.stage[k]);
    if (d.stage_ev[k]) (void)hipEventDestroy(d.stage_ev[k]);
    d.stage[k] = nullptr;
    d.stage_ev[k] = nullptr;
  }
  d.stage_bytes = 0;
  delete d.stage_pool;
  d.stage_pool = nullptr;
  (void)hipFree(d.pair_out);
  d.pair_out = nullptr;
  d.pair_out_cap = 0;
  if (d.copy) (void)hipStreamDestroy(d.copy);
  d.copy = nullptr;
}

namespace {

struct Job {
  const uint8_t* const* frames;
  int n_frames, width, height, stride, blk, range, cost;
  const int* pairs;
  int16_t* mv_xy;
  uint32_t* block_cost;
};

// Make sure the device's pipeline resources fit this frame size.
me_status prepare(me_ctx* c, Dev& d, size_t plane) {
  me_status s0 = own_stream(c, d);
  if (s0 != ME_OK) return s0;
  if (d.slot_bytes != plane) {  // frame size changed: drop the old slots
    HIPCHK(c, hipStreamSynchronize(d.stream));
    if (d.copy) HIPCHK(c, hipStreamSynchronize(d.copy));
    for (size_t i = 0; i < d.slot_chunks.size(); i++) (void)hipFree(d.slot_chunks[i]);
    d.slot_chunks.clear();
    d.slot_spare.clear();
    d.slots.clear();
    d.slot_bytes = plane;
  }
  if (!d.copy) HIPCHK(c, hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
  if (!d.d2h && tuning().stream_d2h == 1) HIPCHK(c, hipStreamCreateWithFlags(&d.d2h, hipStreamNonBlocking));
  for (int k = 0; k < kEvRing; k++) {
    if (!d.upl_ev[k]) HIPCHK(c, hipEventCreateWithFlags(&d.upl_ev[k], hipEventDisableTiming));
    if (!d.batch_ev[k]) HIPCHK(c, hipEventCreateWithFlags(&d.batch_ev[k], hipEventDisableTiming));
    if (!d.d2h_ev[k]) HIPCHK(c, hipEventCreateWithFlags(&d.d2h_ev[k], hipEventDisableTiming));
  }
  if (d.d2h) HIPCHK(c, hipStreamSynchronize(d.d2h));  // a failed earlier call may have left copies
  return ME_OK;
}

// Upload rows [0, H) of a pinned frame (row pitch `stride`) into a slot on the
// copy stream.  Row chunks on extra streams measured slower (H2D at 1080p: 2
// streams 10.5k -> 10.5k pairs/s at best and often 4.7k, 3-4 streams 8.9k at
// best; profiles/r03bm_stream_split_sweep.txt).
me_status upload_pinned(me_ctx* c, Dev& d, uint8_t* dst, const uint8_t* src, int W, int H,
                        int stride) {
  if (stride == W)
    HIPCHK(c, hipMemcpyAsync(dst, src, (size_t)W * H, hipMemcpyHostToDevice, d.copy));
  else
    HIPCHK(c, hipMemcpy2DAsync(dst, W, src, stride, W, H, hipMemcpyHostToDevice, d.copy));
  return ME_OK;
}

// Slots are allocated kSlotChunk at a time, adjacent in one allocation, and
// handed out (and, being freed in upload order, reused) in address order, so
// a batch's new frames mostly land in adjacent slots: frames adjacent in host
// memory too then go up in one copy (upload_batch).
constexpr int kSlotChunk = 8;

me_status new_slot(me_ctx* c, Dev& d, int* idx) {
  if (d.slot_spare.empty()) {
    uint8_t* p = nullptr;
    if (hipMalloc((void**)&p, d.slot_bytes * kSlotChunk) != hipSuccess)
      return fail(c, ME_ENOMEM, "hipMalloc(%zu) for %d frame slots failed", d.slot_bytes * kSlotChunk,
                  kSlotChunk);
    d.slot_chunks.push_back(p);
    for (int k = kSlotChunk - 1; k >= 0; k--) d.slot_spare.push_back(p + (size_t)k * d.slot_bytes);
  }
  d.slots.push_back(d.slot_spare.back());
  d.slot_spare.pop_back();
  *idx = (int)d.slots.size() - 1;
  return ME_OK;
}

me_status ensure_staging(me_ctx* c, Dev& d, size_t plane) {
  if (d.stage_bytes >= plane && d.stage[0]) return ME_OK;
  for (int k = 0; k < 2; k++) {
    if (d.stage_ev[k]) HIPCHK(c, hipEventSynchronize(d.stage_ev[k]));
    if (d.stage[k]) (void)hipHostFree(d.stage[k]);
    d.stage[k] = nullptr;
  }
  d.stage_bytes = 0;
  for (int k = 0; k < 2; k++) {
    if (hipHostMalloc((void**)&d.stage[k], plane, hipHostMallocDefault) != hipSuccess)
      return fail(c, ME_ENOMEM, "pinned staging of %zu bytes failed", plane);
    if (!d.stage_ev[k]) HIPCHK(c, hipEventCreateWithFlags(&d.stage_ev[k], hipEventDisableTiming));
  }
  d.stage_bytes = plane;
  return ME_OK;
}

// Pairs [p0, p1) of the job on device d (the calling thread owns d).
me_status run_pairs(me_ctx* c, Dev& d, const Job& j, int p0, int p1) {
  if (p1 <= p0) return ME_OK;
  HIPCHK(c, hipSetDevice(d.id));
  const int W = j.width, H = j.height, B = j.blk;
  const size_t plane = (size_t)W * H;
  const size_t nb = (size_t)me_num_blocks(W, H, B);
  const int nby = (H + B - 1) / B;
  me_status s = prepare(c, d, plane);
  if (s != ME_OK) return s;
  const size_t np = (size_t)(p1 - p0);
  if ((s = grow(c, (void**)&d.pair_out, &d.pair_out_cap, np * nb * 8)) != ME_OK) return s;
  int16_t* out_mv = reinterpret_cast<int16_t*>(d.pair_out);
  uint32_t* out_cost = reinterpret_cast<uint32_t*>(d.pair_out + np * nb * 4);
  // Pinned bounce buffer for the records: one region of G pairs per batch,
  // indexed by batch mod the region count: one region per batch of this
  // call (the ramp's batches counted exactly) up to kEvRing, and drain()
  // keeps fewer than kEvRing batches between download and drain, so a region
  // is free again when its batch index comes round: at most kEvRing * G
  // pairs pinned, whatever the length of the pair list.  (Round 5 sized it
  // ceil(np / G) + 4, below the ramp's batch count for a large G.)
  bool all_pinned = true;
  for (int n = p0; n < p1 && all_pinned; n++)
    for (int side = 0; side < 2; side++)
      all_pinned = all_pinned &&
                   host_range_pinned(j.frames[j.pairs[2 * n + side]], (size_t)(H - 1) * j.stride + W);
  // pinned frames: 12 pairs per launch (one-ahead uploads); pageable: round 5's 8
  const int G = tuning().stream_batch > 0 ? tuning().stream_batch : all_pinned ? kPairBatch : 8;
  const size_t region = (size_t)G * nb * 8;  // [G * nb mv (4 B)][G * nb cost (4 B)]
  // Batches ramp up 1, 2, 3, 4, 6, 9, then G pairs: the first search starts
  // after two uploads instead of G + 1.  A batch's new frames upload while the
  // batch before it searches, and one upload (42 us at 1080p) is 0.6-0.7 of a
  // pair's search, so batches may grow by about 1.5x: doubling left the GPU
  // idle 27, 55 and 128 us before the 2-, 4- and 8-pair searches
  // (profiles/r04m_*).  (Tuning build: ME_STREAM_GROW = growth in tenths.)
  std::vector<std::pair<int, int>> sched;  // pairs [n0, n1) of each batch
  {
    const int grow = tuning().stream_grow > 0 ? tuning().stream_grow : 5;
    for (int n0 = p0, gb = 1; n0 < p1; n0 += gb, gb = std::min(gb + std::max(1, gb * grow / 10), G)) {
      if (tuning().stream_ramp == 0) gb = G;  // tuning build: fixed batches (the round-3 behaviour)
      sched.emplace_back(n0, std::min(p1, n0 + gb));
    }
  }
  const int nsched = (int)sched.size();
  const size_t nbatches = (size_t)nsched;
  const size_t bneed = region * std::min<size_t>(kEvRing, nbatches);
  if (d.bounce_cap < bneed) {
    if (d.bounce) (void)hipHostFree(d.bounce);
    d.bounce = nullptr;
    d.bounce_cap = 0;
    if (hipHostMalloc((void**)&d.bounce, bneed, hipHostMallocDefault) != hipSuccess)
      return fail(c, ME_ENOMEM, "pinned record buffer of %zu bytes failed", bneed);
    d.bounce_cap = bneed;
  }
  const size_t nregions = d.bounce_cap / region;
  auto bnc_mv = [&](int b) { return reinterpret_cast<int16_t*>(d.bounce + (size_t)(b % nregions) * region); };
  auto bnc_cost = [&](int b) {
    return reinterpret_cast<uint32_t*>(d.bounce + (size_t)(b % nregions) * region + region / 2);
  };
  // Records of batch b leave on the copy stream, queued behind batch b + 1's
  // uploads (which must overlap batch b's search) and ahead of batch b + 2's
  // (which the host enqueues only after batch b is done anyway).  A stream of
  // their own measured the same alone, but one more stream than the process's
  // hardware queues (GPU_MAX_HW_QUEUES = 4: torch's, the caller's, compute,
  // copy) shares a queue with the search or the uploads: 13.0k instead of
  // 14.2k pinned 1080p pairs/s after searches on a torch stream
  // (profiles/r04r_*).  The tuning build's ME_STREAM_D2H=1 restores it.
  const bool own_dl = d.d2h != nullptr;
  hipStream_t dl = own_dl ? d.d2h : d.copy;
  std::vector<std::pair<int, int>> ranges;  // pairs [n0, n1) of each batch
  int downloaded = 0;  // batches whose record copies are enqueued: [0, downloaded)
  auto download = [&]() -> me_status {
    const int b = downloaded++;
    const size_t o = (size_t)(ranges[b].first - p0) * nb;
    const size_t k = (size_t)(ranges[b].second - ranges[b].first) * nb;
    HIPCHK(c, hipStreamWaitEvent(dl, d.batch_ev[b % kEvRing], 0));
    HIPCHK(c, hipMemcpyAsync(bnc_mv(b), out_mv + 2 * o, k * 4, hipMemcpyDeviceToHost, dl));
    if (j.block_cost)
      HIPCHK(c, hipMemcpyAsync(bnc_cost(b), out_cost + o, k * 4, hipMemcpyDeviceToHost, dl));
    HIPCHK(c, hipEventRecord(d.d2h_ev[b % kEvRing], dl));
    return ME_OK;
  };
  // batches whose records the host has moved to the caller: [0, drained)
  int drained = 0;
  auto drain = [&](int upto) -> me_status {  // batches <= upto
    for (; drained <= upto && drained < downloaded; drained++) {
      HIPCHK(c, hipEventSynchronize(d.d2h_ev[drained % kEvRing]));
      const size_t o = (size_t)(ranges[drained].first - p0) * nb;
      const size_t k = (size_t)(ranges[drained].second - ranges[drained].first) * nb;
      memcpy(j.mv_xy + 2 * nb * p0 + 2 * o, bnc_mv(drained), k * 4);
      if (j.block_cost) memcpy(j.block_cost + nb * p0 + o, bnc_cost(drained), k * 4);
    }
    return ME_OK;
  };

  std::vector<int> last_use(j.n_frames, -1), slot_of(j.n_frames, -1);
  for (int n = p0; n < p1; n++) {
    last_use[j.pairs[2 * n]] = n;
    last_use[j.pairs[2 * n + 1]] = n;
  }
  std::deque<int> free_slots;  // oldest-freed first
  for (int i = 0; i < (int)d.slots.size(); i++) free_slots.push_back(i);
  // per slot: the last batch of this call whose search read it (-1: none; the
  // previous call ended with the device idle)
  std::vector<int> last_batch(d.slots.size(), -1);
  int stage_k = 0;
  const size_t span = (size_t)(H - 1) * j.stride + W;

  // The host runs at most kAhead pairs ahead of the GPU.  Unbounded, the host
  // intermittently blocked for 7-10 ms inside an enqueue while the GPU sat idle
  // (1080p pan over 64 pairs, medians of 5: pinned 4.6k pairs/s, worst 3.2k).
  // Bounded (pinned / pageable, 64 pairs): 2 ahead 10.3k / 7.9k, 3 ahead 9.2k /
  // 9.5k, 4 ahead 9.4k / 9.0k.  Pinned frames need the host only to enqueue a
  // pair (~25 us); pageable ones also to copy them into staging, so they get
  // one more pair of slack.
  const int env_ahead = tuning().stream_ahead;  // tuning build: 1..8, 9 unbounded (diagnostic)
  const int kAhead = env_ahead > 8 ? 1 << 30 : env_ahead >= 1 ? env_ahead : (all_pinned ? 2 : 3);
  // Pairs are searched G at a time in one job-table launch (launch_jobs: the
  // flow / item kernels' job tables, SSD pairs sharing the matrix cores'
  // launches), so a launch's fill and drain are paid once per G pairs.  The
  // slots a batch frees cool while later batches' frames upload into older
  // ones.  Uploads run one batch ahead (below): batch b + 1's are enqueued when
  // the host has waited for batch b - 2, so the slots they reuse must have been
  // freed by batch b - 2 or earlier -- two batches' worth cooling, at least
  // 2 G + 1 (with G + 1, most reused slots were batch b - 1's, and the copy
  // queue waited for that search before uploading).
  // (tuning build: ME_STREAM_UPL = U batches ahead needs (U + 1) G + 1)
  // Pageable frames keep round 5's order (a batch's uploads just before its
  // search, U = 0) and 8 pairs per launch: their rate is bound by the host's
  // staging copies, and one-ahead uploads gained nothing there (paired runs,
  // four rounds: 11.6-12.8k one ahead, 11.7-13.0k this way, 11.0-12.6k round
  // 5's code; profiles/r06zn_stream_ab.jsonl).
  const int U = tuning().stream_upl > 0 ? tuning().stream_upl : all_pinned ? 1 : 0;
  const size_t cool = (size_t)std::max(cooling_slots(), (U + 1) * G + 1);
  // Ordering events: one per batch on each stream, not one per frame slot.
  // The round-3 scheme (a ready event per upload, a free event per released
  // slot, one wait per frame of every pair) put ~13 event packets between two
  // search launches on the compute stream and a wait + record around every
  // upload on the copy stream; the trace showed each search starting 58-74 us
  // after the previous one ended although its uploads had landed 150 us
  // earlier, and ~17 us between consecutive uploads (profiles/r04e_*).
  int synced = -1;  // newest batch the host has waited for
  std::vector<SearchJob> jobs;
  jobs.reserve((size_t)G);
  // Uploads run one batch ahead of the searches (round 6): batch b + 1's new
  // frames are enqueued on the copy stream together with batch b's search, so
  // by the time batch b + 1's search is enqueued (the host waits for batch
  // b - 1 first) they have usually landed, and the host, seeing their event
  // complete, enqueues the search with no wait packet on the compute queue.
  // The wait packets were the launch gaps: 18.5 us between launches, and
  // 14.8-15.0k instead of 14.0k pinned pairs/s without them
  // (profiles/r05zz6_stream_wait_experiments.txt).
  std::vector<char> has_upl((size_t)nsched, 0);
  // pinned frames of a batch whose slots and host rows are both adjacent go up
  // in one copy: 2 MB copies ran at 44.7 GB/s against 49.9 for large ones
  // (profiles/r03bp_h2d_probe.txt), ~10 us between back-to-back copies
  // (profiles/r06u_*), and the ramp's growth is bound by the upload rate
  // (one copy never spans two allocations: the slots of one chunk, host rows
  // inside one me_host_alloc range -- adjacent addresses alone are not enough)
  uint8_t* run_dst = nullptr;
  const uint8_t* run_src = nullptr;
  size_t run_n = 0;
  int run_si = -1;
  auto flush_run = [&]() -> me_status {
    if (run_n) {
      me_status st;
      if ((st = upload_pinned(c, d, run_dst, run_src, W, (int)(H * run_n), W)) != ME_OK) return st;
    }
    run_n = 0;
    return ME_OK;
  };
  auto upload_batch = [&](int bi) -> me_status {
    int uploads = 0;
    for (int n = sched[bi].first; n < sched[bi].second; n++) {
      for (int side = 0; side < 2; side++) {
        const int f = j.pairs[2 * n + side];
        if (slot_of[f] >= 0) continue;
        // Keep freed slots cooling: reusing a slot the previous batch just
        // released would serialise this upload behind that search.
        int si;
        me_status st;
        if (free_slots.size() < cool) {
          if ((st = new_slot(c, d, &si)) != ME_OK) return st;
          last_batch.push_back(-1);
        } else {
          si = free_slots.front();
          free_slots.pop_front();
          // its last reader may still run only if the host has not waited for
          // it yet (a later batch's event in the ring covers it too: in order)
          const int lb = last_batch[si];
          if (lb > synced) HIPCHK(c, hipStreamWaitEvent(d.copy, d.batch_ev[lb % kEvRing], 0));
        }
        const uint8_t* src = j.frames[f];
        if (host_range_pinned(src, span)) {
          if (j.stride != W) {
            if ((st = flush_run()) != ME_OK) return st;
            if ((st = upload_pinned(c, d, d.slots[si], src, W, H, j.stride)) != ME_OK) return st;
          } else if (run_n && si == run_si + (int)run_n && si / kSlotChunk == run_si / kSlotChunk &&
                     d.slots[si] == run_dst + run_n * plane && src == run_src + run_n * plane &&
                     host_range_pinned(run_src, (run_n + 1) * plane)) {
            run_n++;
          } else {
            if ((st = flush_run()) != ME_OK) return st;
            run_dst = d.slots[si];
            run_src = src;
            run_si = si;
            run_n = 1;
          }
        } else {
          if ((st = flush_run()) != ME_OK) return st;
          if ((st = ensure_staging(c, d, plane)) != ME_OK) return st;
          // the copy that last read this staging buffer must be done
          HIPCHK(c, hipEventSynchronize(d.stage_ev[stage_k]));
          uint8_t* stg = d.stage[stage_k];
          // The copy into staging is host-memory-bound on one thread (a 1080p
          // frame ~80 us, more than a pair's search): split it over the caller
          // and kCpy - 1 helper threads.
          auto copy_rows = [&](int y0, int y1) {
            if (j.stride == W)
              memcpy(stg + (size_t)y0 * W, src + (size_t)y0 * W, (size_t)(y1 - y0) * W);
            else
              for (int y = y0; y < y1; y++) memcpy(stg + (size_t)y * W, src + (size_t)y * j.stride, W);
          };
          const int kCpy = std::min(tuning().stream_cpy > 0 ? tuning().stream_cpy : 4, std::max(1, H / 64));
          if (kCpy > 1 && !d.stage_pool) {
            try {
              d.stage_pool = new Workers(kCpy - 1);
            } catch (...) {  // no thread could be started: copy on this thread
              d.stage_pool = nullptr;
            }
          }
          if (kCpy > 1 && d.stage_pool && d.stage_pool->size() + 1 >= kCpy)
            d.stage_pool->run_split(kCpy, [&](int i) { copy_rows(H * i / kCpy, H * (i + 1) / kCpy); });
          else
            copy_rows(0, H);
          if ((st = upload_pinned(c, d, d.slots[si], stg, W, H, W)) != ME_OK) return st;
          HIPCHK(c, hipEventRecord(d.stage_ev[stage_k], d.copy));
          stage_k ^= 1;
        }
        uploads++;
        slot_of[f] = si;
      }
    }
    {
      const me_status st = flush_run();
      if (st != ME_OK) return st;
    }
    // one event for this batch's uploads (the copy stream is in order: frames
    // uploaded by earlier batches are covered by their batches' events)
    if (uploads) {
      HIPCHK(c, hipEventRecord(d.upl_ev[bi % kEvRing], d.copy));
      has_upl[bi] = 1;
    }
    return ME_OK;
  };
  int batch = 0;
  for (; batch < nsched; batch++) {
    const int n0 = sched[batch].first, n1 = sched[batch].second;
    if (kAhead <= 8 && batch >= kAhead) {
      HIPCHK(c, hipEventSynchronize(d.batch_ev[(batch - kAhead) % kEvRing]));
      synced = batch - kAhead;
    }
    if (U == 0 && (s = upload_batch(batch)) != ME_OK) return s;
    if (batch == 0)
      for (int u = 0; u < U && u < nsched; u++)
        if ((s = upload_batch(u)) != ME_OK) return s;
    jobs.clear();
    me::SearchArgs base{};
    for (int n = n0; n < n1; n++) {
      const int sr = slot_of[j.pairs[2 * n]], sc = slot_of[j.pairs[2 * n + 1]];
      const size_t o = (size_t)(n - p0) * nb;
      if (n == n0)
        base = make_args(d.slots[sr], 0, d.slots[sc], 0, W, H, W, B, j.range, j.cost, 0, nby,
                         out_mv + 2 * o, out_cost + o);
      jobs.push_back(SearchJob{d.slots[sr], 0, d.slots[sc], 0, 0, nby, out_mv + 2 * o, out_cost + o});
    }
    // this batch's uploads: a wait packet only if they have not landed yet
    if (has_upl[batch]) {
      const hipError_t q = hipEventQuery(d.upl_ev[batch % kEvRing]);
      if (q == hipErrorNotReady)
        HIPCHK(c, hipStreamWaitEvent(d.stream, d.upl_ev[batch % kEvRing], 0));
      else if (q != hipSuccess)
        return fail(c, ME_EDEVICE, "upload event: %s", hipGetErrorString(q));
    }
    if ((s = me::attach_scratch(c, d, base, false, n1 - n0)) != ME_OK) return s;
    if ((s = me::launch_jobs_ordered(c, d, base, jobs.data(), n1 - n0, d.stream)) != ME_OK) return s;
    HIPCHK(c, hipEventRecord(d.batch_ev[batch % kEvRing], d.stream));
    ranges.emplace_back(n0, n1);
    // then the next batch's uploads (after the launch: pageable frames' host
    // copies into staging must not hold back this search's enqueue), then the
    // previous batch's records behind them on the copy stream
    if (U > 0 && batch + U < nsched && (s = upload_batch(batch + U)) != ME_OK) return s;
    while (!own_dl && downloaded < batch)
      if ((s = download()) != ME_OK) return s;
    if (own_dl && (s = download()) != ME_OK) return s;
    // Move the records of batches the host already waited for (their downloads
    // are done or nearly), and never let the event ring wrap.
    if ((s = drain(std::max(synced - 1, batch - kEvRing + 2))) != ME_OK) return s;
    for (int n = n0; n < n1; n++)
      for (int side = 0; side < 2; side++) {
        const int f = j.pairs[2 * n + side];
        if (last_use[f] < n1 && slot_of[f] >= 0) {
          const int si = slot_of[f];
          last_batch[si] = batch;
          free_slots.push_back(si);
          slot_of[f] = -1;
        }
      }
  }
  while (downloaded < batch)
    if ((s = download()) != ME_OK) return s;
  if ((s = drain(batch)) != ME_OK) return s;
  return me::device_status(c, d, d.stream);
}

}  // namespace
}  // namespace me

extern "C" {

void* me_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (bytes == 0 || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(me::g_pin_mu);
  me::g_pinned[(uintptr_t)p] = bytes;
  return p;
}

void me_host_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(me::g_pin_mu);
    if (me::g_pinned.erase((uintptr_t)p) == 0) return;  // not ours
  }
  (void)hipHostFree(p);
}

me_status me_search_pairs(me_ctx* c, const uint8_t* const* frames, int n_frames, int width,
                          int height, int stride, int blk, int range, me_cost cost,
                          const int* pairs, int n_pairs, int16_t* mv_xy, uint32_t* block_cost) {
  if (!c) return ME_EINVAL;
  if (n_pairs < 0 || n_frames < 0) return me::fail(c, ME_EINVAL, "n_pairs %d n_frames %d", n_pairs, n_frames);
  if (n_pairs == 0) return ME_OK;
  if (!frames || !pairs) return me::fail(c, ME_EINVAL, "null frames or pairs");
  for (int n = 0; n < n_pairs; n++)
    for (int side = 0; side < 2; side++) {
      const int f = pairs[2 * n + side];
      if (f < 0 || f >= n_frames) return me::fail(c, ME_EINVAL, "pair %d: frame index %d", n, f);
      if (!frames[f]) return me::fail(c, ME_EINVAL, "frame %d is null", f);
    }
  me_status s = me::check_args(c, frames[pairs[0]], frames[pairs[1]], width, height, stride, blk,
                               range, cost, mv_xy);
  if (s != ME_OK) return s;
  c->err[0] = 0;
  const me::Job job{frames, n_frames, width, height, stride, blk, range, (int)cost, pairs,
                    mv_xy, block_cost};
  const int nd = (int)c->devs.size();
  if (nd == 1) return me::run_pairs(c, c->devs[0], job, 0, n_pairs);
  // One persistent host worker per device, contiguous runs of pairs (shared frames of
  // neighbouring pairs stay on one device); errors land in per-thread contexts.
  me::Workers* pool = me::workers(c);
  if (!pool) return me::fail(c, ME_ENOMEM, "host worker threads");
  std::vector<me_ctx> errs(nd);
  for (me_ctx& e : errs) e.owner = c;
  std::vector<me_status> st(nd, ME_OK);
  pool->run(nd, [&](int i) {
    const int p0 = (int)((long)n_pairs * i / nd), p1 = (int)((long)n_pairs * (i + 1) / nd);
    st[i] = me::run_pairs(&errs[i], c->devs[i], job, p0, p1);
  });
  for (int i = 0; i < nd; i++)
    if (st[i] != ME_OK) return me::fail(c, st[i], "device %d: %s", c->devs[i].id, errs[i].err);
  return ME_OK;
}

}  // extern "C"
