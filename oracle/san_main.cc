// san_main.cc -- CPU sanitizer harness (TEST INFRASTRUCTURE; SURVEY §5 asks
// for the CPU code under TSAN / ASAN).  Built by `make -C oracle asan tsan`
// (tests/test_sanitizers.py runs both), it exercises the host code that runs
// threads or parses untrusted input, without a GPU:
//   - the oracle's pthread pool (orc_full_search: workers pulling block indices
//     from a shared counter), against a single-thread run of the same search;
//   - the stripe planner (me_plan.cpp: me_plan_stripes, me_candidate_count) over
//     many shapes, checking the partition invariants;
//   - the file readers (me_io.cpp) fed truncated, corrupt and hostile files:
//     every one must come back as ME_EIO / ME_EINVAL, never a crash or an
//     out-of-bounds access (the reference's reader never checks its fopen,
//     src/common/utils.c:61-67).
// Exit status 0 and "san ok" on success; the sanitizers abort otherwise.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "me.h"
#include "me_oracle.h"

#define CHECK(x)                                                   \
  do {                                                             \
    if (!(x)) {                                                    \
      fprintf(stderr, "san: check failed at %d: %s\n", __LINE__, #x); \
      exit(1);                                                     \
    }                                                              \
  } while (0)

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64() {  // splitmix64
  uint64_t z = (rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void pool() {
  const int W = 97, H = 61;
  std::vector<uint8_t> ref(W * H), cur(W * H);
  for (int i = 0; i < W * H; i++) {
    ref[i] = (uint8_t)next_u64();
    cur[i] = (uint8_t)(i % 7 == 0 ? ref[i] : next_u64());
  }
  const int kinds[] = {ORC_SSD, ORC_SAD, ORC_MSE_FLOAT};
  for (int kind : kinds)
    for (int blk : {4, 8, 16}) {
      const int n = orc_num_blocks(W, H, blk);
      std::vector<int16_t> mv1(2 * n), mvn(2 * n);
      std::vector<uint32_t> c1(n), cn(n);
      CHECK(orc_full_search(ref.data(), cur.data(), W, H, W, blk, 6, kind, 1, 0, n, mv1.data(),
                            c1.data(), nullptr) == 0);
      // many threads over a small job list: contention on the shared counter
      CHECK(orc_full_search(ref.data(), cur.data(), W, H, W, blk, 6, kind, 13, 0, n, mvn.data(),
                            cn.data(), nullptr) == 0);
      CHECK(mv1 == mvn && c1 == cn);
    }
}

static void planner() {
  for (int t = 0; t < 3000; t++) {
    const int W = 1 + (int)(next_u64() % 4000), H = 1 + (int)(next_u64() % 2500);
    const int blk = 1 + (int)(next_u64() % 64), S = (int)(next_u64() % 300);
    const int n = 1 + (int)(next_u64() % 16);
    std::vector<int> b(n + 1, -1);
    CHECK(me_plan_stripes(W, H, blk, S, n, b.data()) == ME_OK);
    const int nby = (H + blk - 1) / blk;
    CHECK(b[0] == 0 && b[n] == nby);
    for (int i = 0; i < n; i++) CHECK(b[i] <= b[i + 1]);
    (void)me_candidate_count(W, H, blk, S);
  }
  int b[3];
  CHECK(me_plan_stripes(10, 10, 0, 1, 2, b) == ME_EINVAL);
  CHECK(me_plan_stripes(10, 10, 4, 1, 0, b) == ME_EINVAL);
  CHECK(me_plan_stripes(10, 10, 4, 1, 2, nullptr) == ME_EINVAL);
  CHECK(me_candidate_count(352, 288, 8, 12) == 927024ull);
}

static std::string tmp_path(const char* name) {
  const char* d = getenv("TMPDIR");
  return std::string(d && *d ? d : "/tmp") + "/me_san_" + std::to_string(getpid()) + "_" + name;
}

static void write_bytes(const std::string& p, const std::vector<uint8_t>& v) {
  FILE* f = fopen(p.c_str(), "wb");
  CHECK(f);
  if (!v.empty()) CHECK(fwrite(v.data(), 1, v.size(), f) == v.size());
  fclose(f);
}

static void files() {
  const int W = 33, H = 17, B = 8, n_pairs = 3;
  const int nb = me_num_blocks(W, H, B);
  std::vector<int16_t> mv(2 * nb * n_pairs);
  std::vector<uint32_t> co(nb * n_pairs);
  for (auto& x : mv) x = (int16_t)next_u64();
  for (auto& x : co) x = (uint32_t)next_u64();
  const std::string good = tmp_path("good.memv");
  CHECK(me_mv_write(good.c_str(), W, H, B, 5, ME_COST_SAD, nullptr, n_pairs, mv.data(),
                    co.data()) == ME_OK);
  FILE* f = fopen(good.c_str(), "rb");
  CHECK(f);
  std::vector<uint8_t> bytes;
  for (int c; (c = fgetc(f)) != EOF;) bytes.push_back((uint8_t)c);
  fclose(f);
  me_mv_header h;
  std::vector<int> pairs(2 * n_pairs);
  std::vector<int16_t> mv2(mv.size());
  std::vector<uint32_t> co2(co.size());
  CHECK(me_mv_read(good.c_str(), &h, pairs.data(), mv2.data(), co2.data()) == ME_OK);
  CHECK(mv2 == mv && co2 == co);

  const std::string bad = tmp_path("bad.memv");
  // every truncation
  for (size_t len = 0; len < bytes.size(); len++) {
    write_bytes(bad, std::vector<uint8_t>(bytes.begin(), bytes.begin() + len));
    me_mv_header hh;
    CHECK(me_mv_read(bad.c_str(), &hh, pairs.data(), mv2.data(), co2.data()) != ME_OK);
  }
  // corrupt header fields (sizes, counts, flags, magic) and random bytes: the
  // reader may accept a consistent file, but must never write past buffers
  // sized from the good header
  for (int t = 0; t < 400; t++) {
    std::vector<uint8_t> v = bytes;
    const int k = 1 + (int)(next_u64() % 4);
    for (int j = 0; j < k; j++) v[next_u64() % 32] = (uint8_t)next_u64();
    if (t % 5 == 0) v.resize(v.size() + (next_u64() % 64));
    write_bytes(bad, v);
    me_mv_header hh;
    if (me_mv_read_header(bad.c_str(), &hh) != ME_OK) continue;
    const long long nbh = me_num_blocks(hh.width, hh.height, hh.block_size);
    if ((long long)hh.n_pairs * nbh > (long long)nb * n_pairs || hh.n_pairs > (uint32_t)n_pairs)
      continue;  // a caller sizes its buffers from the header it read
    (void)me_mv_read(bad.c_str(), &hh, pairs.data(), mv2.data(), co2.data());
  }
  CHECK(me_mv_read_header(tmp_path("missing.memv").c_str(), &h) == ME_EIO);

  // YUV: a short last frame is not a frame; out-of-range indices are refused
  const std::string yuv = tmp_path("f.yuv");
  std::vector<uint8_t> frames(2 * W * H + W * H / 2);
  for (auto& x : frames) x = (uint8_t)next_u64();
  write_bytes(yuv, frames);
  CHECK(me_yuv_frame_count(yuv.c_str(), W, H, ME_YUV_LUMA) == 2);
  std::vector<uint8_t> dst(W * H);
  CHECK(me_yuv_read_luma(yuv.c_str(), W, H, ME_YUV_LUMA, 1, dst.data(), W) == ME_OK);
  CHECK(memcmp(dst.data(), frames.data() + W * H, W * H) == 0);
  CHECK(me_yuv_read_luma(yuv.c_str(), W, H, ME_YUV_LUMA, 2, dst.data(), W) != ME_OK);
  CHECK(me_yuv_read_luma(yuv.c_str(), W, H, ME_YUV_LUMA, -1, dst.data(), W) != ME_OK);
  CHECK(me_yuv_read_luma(yuv.c_str(), W, H, ME_YUV_I420, 1, dst.data(), W) != ME_OK);
  CHECK(me_yuv_read_luma(yuv.c_str(), 0, H, ME_YUV_LUMA, 0, dst.data(), W) != ME_OK);
  CHECK(me_yuv_frame_count(tmp_path("missing.yuv").c_str(), W, H, ME_YUV_LUMA) == -1);
  unlink(good.c_str());
  unlink(bad.c_str());
  unlink(yuv.c_str());
}

int main() {
  pool();
  planner();
  files();
  printf("san ok\n");
  return 0;
}
