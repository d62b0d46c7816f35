// Layout switches of the feature-sliced multi-GPU SageBlock (sldm_sage/dist.py):
// a rank's rows [rows, W*cs] <-> W column blocks [W][rows][cs] (the buffers
// its all-to-alls send and receive), with the backward's two-term add fused
// into the unpack (dx = dx_root + unpack(dAgg-gradient blocks)).
//
// Pure byte moves, HBM-bound: 2 * rows * W * cs * s bytes per call (+ rows *
// W * cs * s for the addend).  One thread per 16-B vector, consecutive threads
// along a row, so the row-layout side is read / written as whole coalesced
// rows and the block side as cs*s-byte runs (64 B at F = 256, W = 8) -- torch's
// generic permuted copy reaches ~3.2 TB/s on these shapes (tools/perm_probe.py),
// a plain copy ~5.3.
#include "common.hpp"

namespace {

constexpr int kBlock = 256;

template <typename T, int V, bool PACK, bool ADD>
__global__ __launch_bounds__(kBlock) void cols_layout_kernel(
    const T* __restrict__ src, int64_t ld_rows, T* __restrict__ dst, int64_t rows, int nblk,
    int cs, const T* __restrict__ addend, int64_t lda) {
  const int vpr = nblk * cs / V;                               // vectors per row
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= rows * vpr) return;
  const int64_t r = i / vpr;
  const int f = (int)(i - r * vpr) * V;                        // column in the row layout
  const int c = f / cs, o = f - c * cs;                        // block, offset in block
  const int64_t bidx = ((int64_t)c * rows + r) * cs + o;       // element in [W][rows][cs]
  if constexpr (PACK) {
    *reinterpret_cast<uint4*>(dst + bidx) = *reinterpret_cast<const uint4*>(src + r * ld_rows + f);
  } else if constexpr (!ADD) {
    *reinterpret_cast<uint4*>(dst + r * ld_rows + f) = *reinterpret_cast<const uint4*>(src + bidx);
  } else {
    float a[V], b[V];
    sldm::Vec<T, V>::load(addend + r * lda + f, a);
    sldm::Vec<T, V>::load(src + bidx, b);
#pragma unroll
    for (int v = 0; v < V; ++v) a[v] = a[v] + b[v];
    sldm::Vec<T, V>::store(dst + r * ld_rows + f, a);
  }
}

template <typename T, bool PACK, bool ADD>
int launch(const void* src, int64_t ld_rows, void* dst, int64_t rows, int nblk, int cs,
           const void* addend, int64_t lda, hipStream_t stream) {
  constexpr int V = 16 / (int)sizeof(T);
  const int64_t n = rows * (int64_t)nblk * cs / V;
  const int64_t grid = (n + kBlock - 1) / kBlock;
  SLDM_REQUIRE(grid < ((int64_t)1 << 31), "sldm cols layout: grid too large");
  cols_layout_kernel<T, V, PACK, ADD><<<(unsigned)grid, kBlock, 0, stream>>>(
      reinterpret_cast<const T*>(src), ld_rows, reinterpret_cast<T*>(dst), rows, nblk, cs,
      reinterpret_cast<const T*>(addend), lda);
  SLDM_LAUNCH_CHECK("cols_layout_kernel");
  return SLDM_OK;
}

int check(int dtype, const void* a, const void* b, int64_t rows, int64_t nblk, int64_t cs,
          int64_t ld_rows, const void* addend, int64_t lda) {
  SLDM_REQUIRE(dtype == SLDM_F32 || dtype == SLDM_BF16, "sldm cols layout: dtype %d", dtype);
  const int v = dtype == SLDM_F32 ? 4 : 8;
  SLDM_REQUIRE(rows >= 0 && nblk >= 1 && cs >= 1 && cs % v == 0 && ld_rows >= nblk * cs &&
                   ld_rows % v == 0 && (!addend || (lda >= nblk * cs && lda % v == 0)),
               "sldm cols layout: needs 16-B column blocks (cs %% %d == 0) and row strides", v);
  const uintptr_t al = 15;
  SLDM_REQUIRE(rows == 0 || (a && b && !(reinterpret_cast<uintptr_t>(a) & al) &&
                             !(reinterpret_cast<uintptr_t>(b) & al) &&
                             !(reinterpret_cast<uintptr_t>(addend) & al)),
               "sldm cols layout: NULL or misaligned pointer");
  return SLDM_OK;
}

}  // namespace

extern "C" int sldm_cols_pack(int dtype, const void* rows_src, int64_t ld_rows, int64_t num_rows,
                              int64_t num_blocks, int64_t block_cols, void* blocks_dst,
                              void* stream_) {
  const int rc = check(dtype, rows_src, blocks_dst, num_rows, num_blocks, block_cols, ld_rows,
                       nullptr, 0);
  if (rc != SLDM_OK || num_rows == 0) return rc;
  hipStream_t s = sldm::as_stream(stream_);
  return dtype == SLDM_F32
             ? launch<float, true, false>(rows_src, ld_rows, blocks_dst, num_rows,
                                          (int)num_blocks, (int)block_cols, nullptr, 0, s)
             : launch<uint16_t, true, false>(rows_src, ld_rows, blocks_dst, num_rows,
                                             (int)num_blocks, (int)block_cols, nullptr, 0, s);
}

extern "C" int sldm_cols_unpack(int dtype, const void* blocks_src, int64_t num_rows,
                                int64_t num_blocks, int64_t block_cols, const void* addend,
                                int64_t ld_add, void* rows_dst, int64_t ld_rows, void* stream_) {
  const int rc = check(dtype, blocks_src, rows_dst, num_rows, num_blocks, block_cols, ld_rows,
                       addend, ld_add);
  if (rc != SLDM_OK || num_rows == 0) return rc;
  hipStream_t s = sldm::as_stream(stream_);
  const int nb = (int)num_blocks, cs = (int)block_cols;
  if (dtype == SLDM_F32)
    return addend ? launch<float, false, true>(blocks_src, ld_rows, rows_dst, num_rows, nb, cs,
                                               addend, ld_add, s)
                  : launch<float, false, false>(blocks_src, ld_rows, rows_dst, num_rows, nb, cs,
                                                nullptr, 0, s);
  return addend ? launch<uint16_t, false, true>(blocks_src, ld_rows, rows_dst, num_rows, nb, cs,
                                                addend, ld_add, s)
                : launch<uint16_t, false, false>(blocks_src, ld_rows, rows_dst, num_rows, nb, cs,
                                                 nullptr, 0, s);
}
