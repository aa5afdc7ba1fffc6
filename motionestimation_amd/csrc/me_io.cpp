// me_io.cpp -- host file formats of the engine (include/me.h).
//
// YUV planes stay u8 end to end: the reference reads a file into u8 and widens
// it to int32 (src/common/utils.c:49-59 yuvReadFrame / copyToIntBuffer) and
// narrows it back on write (utils.c:61-92); here planes are read straight
// into the caller's u8 buffer, at any frame index of a multi-frame file.
// The MV-field file is this build's own format (the reference never writes
// its MVs): a 32-byte header and, per pair, the raster-order MV records and
// optional costs, little-endian.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "me.h"

namespace {

struct File {
  FILE* f;
  explicit File(FILE* x) : f(x) {}
  ~File() {
    if (f) fclose(f);
  }
};

int64_t frame_bytes(int width, int height, me_yuv_layout layout) {
  const int64_t luma = (int64_t)width * height;
  return layout == ME_YUV_I420 ? luma + 2 * (((int64_t)width + 1) / 2) * ((height + 1) / 2) : luma;
}

int64_t file_size(FILE* f) {
  if (fseeko(f, 0, SEEK_END) != 0) return -1;
  const int64_t n = (int64_t)ftello(f);
  if (fseeko(f, 0, SEEK_SET) != 0) return -1;
  return n;
}

bool bad_geometry(int width, int height, me_yuv_layout layout) {
  return width <= 0 || height <= 0 || (layout != ME_YUV_LUMA && layout != ME_YUV_I420);
}

// Bytes one pair occupies in the file (indices, MV records, costs).
int64_t pair_bytes(const me_mv_header& h) {
  const int64_t nb = me_num_blocks(h.width, h.height, h.block_size);
  return 8 + nb * ((h.flags & 1) ? 8 : 4);
}

bool valid_header(const me_mv_header& h) {
  if (!(memcmp(h.magic, "MEMV", 4) == 0 && h.version == 1 && h.flags <= 1 && h.width > 0 &&
        h.height > 0 && h.block_size > 0 && h.block_size <= ME_MAX_BLOCK &&
        h.search_range >= 0 &&
        (h.cost == ME_COST_SSD || h.cost == ME_COST_SAD || h.cost == ME_COST_SSIM)))
    return false;
  // the block count fits an int and the whole file an int64 (hostile headers)
  if (me_num_blocks(h.width, h.height, h.block_size) <= 0) return false;
  return (int64_t)h.n_pairs <= (INT64_MAX - 32) / pair_bytes(h);
}

}  // namespace

extern "C" {

int64_t me_yuv_frame_count(const char* path, int width, int height, me_yuv_layout layout) {
  if (!path || bad_geometry(width, height, layout)) return -1;
  File f(fopen(path, "rb"));
  if (!f.f) return -1;
  const int64_t n = file_size(f.f);
  return n < 0 ? -1 : n / frame_bytes(width, height, layout);
}

me_status me_yuv_read_luma(const char* path, int width, int height, me_yuv_layout layout,
                           int frame_index, uint8_t* dst, int dst_stride) {
  if (!path || !dst || bad_geometry(width, height, layout) || frame_index < 0 ||
      dst_stride < width)
    return ME_EINVAL;
  File f(fopen(path, "rb"));
  if (!f.f) return ME_EIO;
  const int64_t fb = frame_bytes(width, height, layout);
  if ((int64_t)frame_index > (INT64_MAX - fb) / fb) return ME_EIO;  // past any file
  const int64_t off = fb * frame_index;
  if (fseeko(f.f, (off_t)off, SEEK_SET) != 0) return ME_EIO;
  if (dst_stride == width)
    return fread(dst, (size_t)width * height, 1, f.f) == 1 ? ME_OK : ME_EIO;
  for (int y = 0; y < height; y++)
    if (fread(dst + (size_t)y * dst_stride, (size_t)width, 1, f.f) != 1) return ME_EIO;
  return ME_OK;
}

me_status me_yuv_write(const char* path, const uint8_t* data, size_t bytes, int append) {
  if (!path || (!data && bytes)) return ME_EINVAL;
  File f(fopen(path, append ? "ab" : "wb"));
  if (!f.f) return ME_EIO;
  if (bytes && fwrite(data, bytes, 1, f.f) != 1) return ME_EIO;
  return fflush(f.f) == 0 ? ME_OK : ME_EIO;
}

me_status me_mv_write(const char* path, int width, int height, int block_size, int search_range,
                      me_cost cost, const int* pairs, int n_pairs, const int16_t* mv_xy,
                      const uint32_t* block_cost) {
  if (!path || n_pairs < 0 || (n_pairs > 0 && !mv_xy)) return ME_EINVAL;
  me_mv_header h;
  memcpy(h.magic, "MEMV", 4);
  h.version = 1;
  h.flags = block_cost ? 1 : 0;
  h.width = width;
  h.height = height;
  h.block_size = block_size;
  h.search_range = search_range;
  h.cost = (int32_t)cost;
  h.n_pairs = (uint32_t)n_pairs;
  if (!valid_header(h)) return ME_EINVAL;
  static_assert(sizeof(me_mv_header) == 32, "header layout");
  const size_t nb = (size_t)me_num_blocks(width, height, block_size);
  File f(fopen(path, "wb"));
  if (!f.f) return ME_EIO;
  if (fwrite(&h, sizeof h, 1, f.f) != 1) return ME_EIO;
  for (int n = 0; n < n_pairs; n++) {
    const int32_t idx[2] = {pairs ? pairs[2 * n] : n, pairs ? pairs[2 * n + 1] : n + 1};
    if (fwrite(idx, sizeof idx, 1, f.f) != 1) return ME_EIO;
    if (nb && fwrite(mv_xy + 2 * nb * n, nb * 4, 1, f.f) != 1) return ME_EIO;
    if (block_cost && nb && fwrite(block_cost + nb * n, nb * 4, 1, f.f) != 1) return ME_EIO;
  }
  return fflush(f.f) == 0 ? ME_OK : ME_EIO;
}

static me_status read_header(FILE* f, me_mv_header* h) {
  if (fread(h, sizeof *h, 1, f) != 1) return ME_EIO;
  return valid_header(*h) ? ME_OK : ME_EIO;
}

me_status me_mv_read_header(const char* path, me_mv_header* hdr) {
  if (!path || !hdr) return ME_EINVAL;
  File f(fopen(path, "rb"));
  if (!f.f) return ME_EIO;
  return read_header(f.f, hdr);
}

me_status me_mv_read(const char* path, me_mv_header* hdr, int* pairs, int16_t* mv_xy,
                     uint32_t* block_cost) {
  if (!path) return ME_EINVAL;
  File f(fopen(path, "rb"));
  if (!f.f) return ME_EIO;
  me_mv_header h;
  me_status s = read_header(f.f, &h);
  if (s != ME_OK) return s;
  if (hdr) *hdr = h;
  const size_t nb = (size_t)me_num_blocks(h.width, h.height, h.block_size);
  const bool has_cost = h.flags & 1;
  // Size check before any read: a truncated file is an error, not a short result.
  const int64_t size = file_size(f.f);
  const int64_t need = (int64_t)sizeof h + (int64_t)h.n_pairs * pair_bytes(h);  // valid_header: no overflow
  if (size != need) return ME_EIO;
  if (fseeko(f.f, (off_t)sizeof h, SEEK_SET) != 0) return ME_EIO;
  for (uint32_t n = 0; n < h.n_pairs; n++) {
    int32_t idx[2];
    if (fread(idx, sizeof idx, 1, f.f) != 1) return ME_EIO;
    if (pairs) {
      pairs[2 * n] = idx[0];
      pairs[2 * n + 1] = idx[1];
    }
    if (mv_xy) {
      if (nb && fread(mv_xy + 2 * nb * n, nb * 4, 1, f.f) != 1) return ME_EIO;
    } else if (fseeko(f.f, (off_t)(nb * 4), SEEK_CUR) != 0) {
      return ME_EIO;
    }
    if (has_cost) {
      if (block_cost) {
        if (nb && fread(block_cost + nb * n, nb * 4, 1, f.f) != 1) return ME_EIO;
      } else if (fseeko(f.f, (off_t)(nb * 4), SEEK_CUR) != 0) {
        return ME_EIO;
      }
    }
  }
  return ME_OK;
}

}  // extern "C"
