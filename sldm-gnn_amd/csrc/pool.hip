// Graph-level readout after the SageBlock: global mean / max pooling over
// the PyG `batch` vector.
//
// Replaces (grusage.py:119-127, :185): PyG 2.7.0 global_mean_pool(x, batch)
// = utils.scatter(x, batch, reduce='mean') and global_max_pool(x, batch) =
// utils.scatter(..., reduce='max'), which on the reference's CPU path is
//   zeros(B, F).scatter_reduce_(0, batch, x, 'amax', include_self=False)
// and, for 'double' pooling, their concatenation.
//
// The batch vector arrives as a segment CSR (seg_rowptr [B+1], member ids in
// ascending node order: the order scatter_add_ visits them).  Segments are cut
// into pieces of at most kPiece rows so one huge segment (a single
// full-graph batch) still spreads over the chip:
//   pool_piece_kernel   per piece: fp32 sum, max and tie count, rows in order
//   pool_finish_kernel  per segment: pieces combined in order -> mean, max and
//                       the max-gradient divisor (below)
//   pool_bwd_kernel     per node: dx = dmean/count + [x == max] dmax/divisor
// A segment of <= kPiece rows is summed strictly in member order, so its mean
// is bit-identical to the reference's fp32 scatter_add_ / count; longer ones
// add per-piece sums in piece order (fp32 rounding only).
//
// Max gradient (torch scatter_reduce backward for amax, what PyG's CPU path
// differentiates): the gradient of a segment/column is split evenly among the
// members equal to the max, and the divisor also counts the zero-initialised
// `self` entry whenever the max equals 0 (self == result there although
// include_self=False).  The divisor stored here is ties + (max == 0).
//
// Algorithmic bytes: forward N*F*s (x) + B*F*(s or 2s) + small partials;
// backward 2*N*F*s + B*F*(3s + 4).
#include "common.hpp"

namespace {

constexpr int kBlock = 256;
constexpr int kPoolPiece = 256;   // rows per piece (one row group each)


template <typename T, int V, int NCH>
__global__ __launch_bounds__(kBlock) void pool_piece_kernel(
    const T* __restrict__ x, int64_t ldx, const int32_t* __restrict__ seg_rowptr,
    const int32_t* __restrict__ member, const int32_t* __restrict__ piece_ptr,
    int64_t num_segments, int64_t num_pieces, int feat, int lpr_log2,
    float* __restrict__ psum, float* __restrict__ pmax, int32_t* __restrict__ pcnt,
    int32_t* __restrict__ parg) {
  const int lpr = 1 << lpr_log2;
  const int lane_in_row = threadIdx.x & (lpr - 1);
  const int64_t piece = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lpr_log2;
  if (piece >= num_pieces) return;
  // segment of this piece: last s with piece_ptr[s] <= piece
  int64_t lo = 0, hi = num_segments;   // piece_ptr[lo] <= piece < piece_ptr[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (piece_ptr[mid] <= piece) lo = mid; else hi = mid;
  }
  const int64_t seg = lo;
  const int beg = seg_rowptr[seg] + (int)(piece - piece_ptr[seg]) * kPoolPiece;
  const int end = min(beg + kPoolPiece, seg_rowptr[seg + 1]);

  int f0[NCH];
  bool act[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int f = (lane_in_row + c * lpr) * V;
    act[c] = f < feat;
    f0[c] = act[c] ? f : feat - V;
  }
  float s[NCH][V], m[NCH][V];
  int n[NCH][V], arg[NCH][V];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int v = 0; v < V; ++v) { s[c][v] = 0.f; m[c][v] = -INFINITY; n[c][v] = 0; arg[c][v] = -1; }

  // running sum, max, tie count and first row holding the max (NaN sticks,
  // as torch's amax; a NaN seen first stays the max)
  auto take = [&](const float (&d)[NCH][V], int row) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float a = d[c][v];
        s[c][v] += a;
        if ((a > m[c][v] || (a != a && m[c][v] == m[c][v])) || arg[c][v] < 0) {
          m[c][v] = a; n[c][v] = 1; arg[c][v] = row;
        } else if (a == m[c][v]) {
          n[c][v] += 1;
        }
      }
  };
  int k = beg;
  for (; k + 4 <= end; k += 4) {   // 4 member rows in flight, consumed in order
    float d[4][NCH][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t r = member[k + u];
#pragma unroll
      for (int c = 0; c < NCH; ++c) sldm::Vec<T, V>::load(x + r * ldx + f0[c], d[u][c]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) take(d[u], member[k + u]);
  }
  for (; k < end; ++k) {
    float d[NCH][V];
    const int64_t r = member[k];
#pragma unroll
    for (int c = 0; c < NCH; ++c) sldm::Vec<T, V>::load(x + r * ldx + f0[c], d[c]);
    take(d, (int)r);
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (!act[c]) continue;
    const int64_t o = piece * (int64_t)feat + f0[c];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      psum[o + v] = s[c][v];
      pmax[o + v] = m[c][v];
      pcnt[o + v] = n[c][v];
      parg[o + v] = arg[c][v];
    }
  }
}

template <typename T, int V, int NCH>
__global__ __launch_bounds__(kBlock) void pool_finish_kernel(
    const int32_t* __restrict__ seg_rowptr, const int32_t* __restrict__ piece_ptr,
    int64_t num_segments, int feat, int lpr_log2, const float* __restrict__ psum,
    const float* __restrict__ pmax, const int32_t* __restrict__ pcnt,
    const int32_t* __restrict__ parg, T* __restrict__ mean_out, int64_t ld_mean,
    T* __restrict__ max_out, int64_t ld_max, float* __restrict__ ndist,
    int32_t* __restrict__ argmax) {
  const int lpr = 1 << lpr_log2;
  const int lane_in_row = threadIdx.x & (lpr - 1);
  const int64_t seg = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lpr_log2;
  if (seg >= num_segments) return;
  const int cnt = seg_rowptr[seg + 1] - seg_rowptr[seg];
  const int p0 = piece_ptr[seg], p1 = piece_ptr[seg + 1];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int f = (lane_in_row + c * lpr) * V;
    if (f >= feat) continue;
    float s[V], m[V], n[V];
    int a[V];
#pragma unroll
    for (int v = 0; v < V; ++v) { s[v] = 0.f; m[v] = -INFINITY; n[v] = 0.f; a[v] = -1; }
    for (int p = p0; p < p1; ++p) {   // pieces in member order: the earlier max wins ties
      const int64_t o = (int64_t)p * feat + f;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float pm = pmax[o + v];
        const float pn = (float)pcnt[o + v];
        s[v] = p == p0 ? psum[o + v] : s[v] + psum[o + v];
        if (p == p0 || pm > m[v] || (pm != pm && m[v] == m[v])) {
          m[v] = pm; n[v] = pn; a[v] = parg[o + v];
        } else if (pm == m[v]) {
          n[v] += pn;
        }
      }
    }
    float mean[V], mx[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      // empty segment: both 0 (zeros(B,F) output; count clamped to 1)
      mean[v] = s[v] / (float)(cnt > 0 ? cnt : 1);
      mx[v] = cnt > 0 ? m[v] : 0.f;
    }
    if (mean_out) sldm::Vec<T, V>::store(mean_out + seg * ld_mean + f, mean);
    if (max_out) sldm::Vec<T, V>::store(max_out + seg * ld_max + f, mx);
    if (ndist) {
      // the divisor tests the stored (dtype-rounded) max against 0, as torch does
#pragma unroll
      for (int v = 0; v < V; ++v)
        ndist[seg * (int64_t)feat + f + v] = n[v] + (sldm::stored_value<T>(mx[v]) == 0.f ? 1.f : 0.f);
    }
    if (argmax) {
#pragma unroll
      for (int v = 0; v < V; ++v) argmax[seg * (int64_t)feat + f + v] = a[v];
    }
  }
}

template <typename T, int V, int NCH>
__global__ __launch_bounds__(kBlock) void pool_bwd_kernel(
    const T* __restrict__ x, int64_t ldx, const int64_t* __restrict__ seg_of,
    const int32_t* __restrict__ seg_rowptr, int64_t num_nodes, int feat, int lpr_log2,
    const T* __restrict__ dmean, int64_t ld_dmean, const T* __restrict__ max_out, int64_t ld_max,
    const T* __restrict__ dmax, int64_t ld_dmax, const float* __restrict__ ndist,
    const int32_t* __restrict__ argmax, T* __restrict__ dx, int64_t ld_dx) {
  const int lpr = 1 << lpr_log2;
  const int lane_in_row = threadIdx.x & (lpr - 1);
  const int64_t row = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lpr_log2;
  if (row >= num_nodes) return;
  const int64_t seg = seg_of[row];
  const int cnt = seg_rowptr[seg + 1] - seg_rowptr[seg];
  const float fc = (float)(cnt > 0 ? cnt : 1);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int f = (lane_in_row + c * lpr) * V;
    if (f >= feat) continue;
    float g[V];
#pragma unroll
    for (int v = 0; v < V; ++v) g[v] = 0.f;
    if (dmean) {
      float dm[V];
      sldm::Vec<T, V>::load(dmean + seg * ld_dmean + f, dm);
#pragma unroll
      for (int v = 0; v < V; ++v) g[v] = dm[v] / fc;
    }
    if (dmax && argmax) {
      // first-argmax routing (x.max(dim) backward: the whole gradient to the
      // first row holding the max)
      float dv[V];
      sldm::Vec<T, V>::load(dmax + seg * ld_dmax + f, dv);
#pragma unroll
      for (int v = 0; v < V; ++v)
        g[v] = g[v] + (argmax[seg * (int64_t)feat + f + v] == (int32_t)row ? dv[v] : 0.f);
    } else if (dmax) {
      float xv[V], mv[V], dv[V];
      sldm::Vec<T, V>::load(x + row * ldx + f, xv);
      sldm::Vec<T, V>::load(max_out + seg * ld_max + f, mv);
      sldm::Vec<T, V>::load(dmax + seg * ld_dmax + f, dv);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float share = dv[v] / ndist[seg * (int64_t)feat + f + v];
        g[v] = g[v] + (xv[v] == mv[v] ? share : 0.f);
      }
    }
    sldm::Vec<T, V>::store(dx + row * ld_dx + f, g);
  }
}

struct Geom { int v, lpr_log2, nch; };

Geom geom(int elem, int64_t feat, std::initializer_list<int64_t> lds,
          std::initializer_list<const void*> ptrs) {
  Geom g;
  g.v = sldm::pick_vec(elem, feat, lds, ptrs);
  const int lpr = sldm::lanes_per_row(feat, g.v);
  g.lpr_log2 = 0;
  while ((1 << g.lpr_log2) < lpr) ++g.lpr_log2;
  g.nch = (int)((feat + (int64_t)lpr * g.v - 1) / ((int64_t)lpr * g.v));
  return g;
}

template <typename T, int V, int NCH>
int launch_fwd(const Geom& g, const T* x, int64_t ldx, const int32_t* seg_rowptr,
               const int32_t* member, const int32_t* piece_ptr, int64_t nseg, int64_t npieces,
               int feat, T* mean_out, int64_t ld_mean, T* max_out, int64_t ld_max, float* ndist,
               int32_t* argmax, float* psum, float* pmax, int32_t* pcnt, int32_t* parg,
               hipStream_t stream) {
  if (npieces > 0) {
    const int64_t grid = ((npieces << g.lpr_log2) + kBlock - 1) / kBlock;
    pool_piece_kernel<T, V, NCH><<<(unsigned)grid, kBlock, 0, stream>>>(
        x, ldx, seg_rowptr, member, piece_ptr, nseg, npieces, feat, g.lpr_log2, psum, pmax, pcnt,
        parg);
    SLDM_LAUNCH_CHECK("pool_piece_kernel");
  }
  const int64_t grid = ((nseg << g.lpr_log2) + kBlock - 1) / kBlock;
  pool_finish_kernel<T, V, NCH><<<(unsigned)grid, kBlock, 0, stream>>>(
      seg_rowptr, piece_ptr, nseg, feat, g.lpr_log2, psum, pmax, pcnt, parg, mean_out, ld_mean,
      max_out, ld_max, ndist, argmax);
  SLDM_LAUNCH_CHECK("pool_finish_kernel");
  return SLDM_OK;
}

template <typename T, int V, int NCH>
int launch_bwd(const Geom& g, const T* x, int64_t ldx, const int64_t* seg_of,
               const int32_t* seg_rowptr, int64_t n, int feat, const T* dmean, int64_t ld_dmean,
               const T* mx, int64_t ld_max, const T* dmax, int64_t ld_dmax, const float* ndist,
               const int32_t* argmax, T* dx, int64_t ld_dx, hipStream_t stream) {
  const int64_t grid = ((n << g.lpr_log2) + kBlock - 1) / kBlock;
  pool_bwd_kernel<T, V, NCH><<<(unsigned)grid, kBlock, 0, stream>>>(
      x, ldx, seg_of, seg_rowptr, n, feat, g.lpr_log2, dmean, ld_dmean, mx, ld_max, dmax, ld_dmax,
      ndist, argmax, dx, ld_dx);
  SLDM_LAUNCH_CHECK("pool_bwd_kernel");
  return SLDM_OK;
}

// (V, NCH) dispatch: V in {8 (bf16 only), 4, 2, 1}, NCH in {1, 2, 4}.
#define SLDM_POOL_DISPATCH(T, g, CALL)                                              \
  do {                                                                              \
    switch ((g).v * 8 + (g).nch) {                                                  \
      case 8 * 8 + 1: if constexpr (sizeof(T) == 2) { return CALL(8, 1); } break;   \
      case 8 * 8 + 2: if constexpr (sizeof(T) == 2) { return CALL(8, 2); } break;   \
      case 8 * 8 + 4: if constexpr (sizeof(T) == 2) { return CALL(8, 4); } break;   \
      case 4 * 8 + 1: return CALL(4, 1);                                            \
      case 4 * 8 + 2: return CALL(4, 2);                                            \
      case 4 * 8 + 4: return CALL(4, 4);                                            \
      case 2 * 8 + 1: return CALL(2, 1);                                            \
      case 2 * 8 + 2: return CALL(2, 2);                                            \
      case 2 * 8 + 4: return CALL(2, 4);                                            \
      case 1 * 8 + 1: return CALL(1, 1);                                            \
      case 1 * 8 + 2: return CALL(1, 2);                                            \
      case 1 * 8 + 4: return CALL(1, 4);                                            \
      default: break;                                                               \
    }                                                                               \
    sldm::set_error("sldm pooling: feature width unsupported (vec %d, chunks %d)",  \
                    (g).v, (g).nch);                                                \
    return SLDM_ERR_ARG;                                                            \
  } while (0)

template <typename T>
int pool_fwd_t(const void* x_, int64_t ldx, const int32_t* seg_rowptr, const int32_t* member,
               const int32_t* piece_ptr, int64_t nseg, int64_t npieces, int64_t feat,
               void* mean_, int64_t ld_mean, void* max_, int64_t ld_max, float* ndist,
               int32_t* argmax, float* psum, float* pmax, int32_t* pcnt, int32_t* parg,
               hipStream_t stream) {
  const T* x = reinterpret_cast<const T*>(x_);
  T* mean_out = reinterpret_cast<T*>(mean_);
  T* max_out = reinterpret_cast<T*>(max_);
  const Geom g = geom((int)sizeof(T), feat,
                      {ldx, mean_out ? ld_mean : 0, max_out ? ld_max : 0}, {x, mean_out, max_out});
#define SLDM_FWD_CALL(VV, NN)                                                             \
  launch_fwd<T, VV, NN>(g, x, ldx, seg_rowptr, member, piece_ptr, nseg, npieces, (int)feat, \
                        mean_out, ld_mean, max_out, ld_max, ndist, argmax, psum, pmax, pcnt, \
                        parg, stream)
  SLDM_POOL_DISPATCH(T, g, SLDM_FWD_CALL);
#undef SLDM_FWD_CALL
}

template <typename T>
int pool_bwd_t(const void* x_, int64_t ldx, const int64_t* seg_of, const int32_t* seg_rowptr,
               int64_t n, int64_t feat, const void* dmean_, int64_t ld_dmean, const void* max_,
               int64_t ld_max, const void* dmax_, int64_t ld_dmax, const float* ndist,
               const int32_t* argmax, void* dx_, int64_t ld_dx, hipStream_t stream) {
  const T* x = reinterpret_cast<const T*>(x_);
  const T* dmean = reinterpret_cast<const T*>(dmean_);
  const T* mx = reinterpret_cast<const T*>(max_);
  const T* dmax = reinterpret_cast<const T*>(dmax_);
  T* dx = reinterpret_cast<T*>(dx_);
  const Geom g = geom((int)sizeof(T), feat,
                      {dmax ? ldx : 0, dmean ? ld_dmean : 0, dmax ? ld_max : 0,
                       dmax ? ld_dmax : 0, ld_dx},
                      {dmax ? x : nullptr, dmean, mx, dmax, dx});
#define SLDM_BWD_CALL(VV, NN)                                                              \
  launch_bwd<T, VV, NN>(g, x, ldx, seg_of, seg_rowptr, n, (int)feat, dmean, ld_dmean, mx,   \
                        ld_max, dmax, ld_dmax, ndist, argmax, dx, ld_dx, stream)
  SLDM_POOL_DISPATCH(T, g, SLDM_BWD_CALL);
#undef SLDM_BWD_CALL
}

}  // namespace

extern "C" int sldm_segment_pool_piece_rows(void) { return kPoolPiece; }

extern "C" size_t sldm_segment_pool_workspace_bytes(int64_t num_pieces, int64_t feat) {
  if (num_pieces <= 0 || feat <= 0) return 256;
  return (size_t)num_pieces * (size_t)feat * 16 + 4 * 256;
}

extern "C" int sldm_segment_pool(int dtype, const void* x, int64_t ldx, const int32_t* seg_rowptr,
                                 const int32_t* member, int64_t num_segments,
                                 const int32_t* piece_ptr, int64_t num_pieces, int64_t feat,
                                 void* mean_out, int64_t ld_mean, void* max_out, int64_t ld_max,
                                 float* max_divisor, int32_t* max_first_row, void* workspace,
                                 size_t workspace_bytes, void* stream_) {
  SLDM_REQUIRE(dtype == SLDM_F32 || dtype == SLDM_BF16, "sldm_segment_pool: dtype %d", dtype);
  SLDM_REQUIRE(num_segments >= 0 && num_pieces >= 0 && feat >= 0 && feat <= 4096,
               "sldm_segment_pool: bad sizes");
  if (num_segments == 0 || feat == 0) return SLDM_OK;
  SLDM_REQUIRE(seg_rowptr && piece_ptr && (num_pieces == 0 || (x && member)),
               "sldm_segment_pool: NULL argument");
  SLDM_REQUIRE(mean_out || max_out, "sldm_segment_pool: neither mean nor max requested");
  SLDM_REQUIRE(!mean_out || ld_mean >= feat, "sldm_segment_pool: ld_mean < feat");
  SLDM_REQUIRE(!max_out || ld_max >= feat, "sldm_segment_pool: ld_max < feat");
  SLDM_REQUIRE(num_pieces == 0 || ldx >= feat, "sldm_segment_pool: ldx < feat");
  const size_t need = sldm_segment_pool_workspace_bytes(num_pieces, feat);
  SLDM_REQUIRE(workspace && workspace_bytes >= need,
               "sldm_segment_pool: workspace too small (%zu < %zu)", workspace_bytes, need);
  auto al = [](uintptr_t p) { return (p + 255) & ~(uintptr_t)255; };
  const size_t plane = (size_t)(num_pieces > 0 ? num_pieces : 1) * (size_t)feat;
  float* psum = reinterpret_cast<float*>(al(reinterpret_cast<uintptr_t>(workspace)));
  float* pmax = reinterpret_cast<float*>(al(reinterpret_cast<uintptr_t>(psum + plane)));
  int32_t* pcnt = reinterpret_cast<int32_t*>(al(reinterpret_cast<uintptr_t>(pmax + plane)));
  int32_t* parg = reinterpret_cast<int32_t*>(al(reinterpret_cast<uintptr_t>(pcnt + plane)));
  hipStream_t stream = sldm::as_stream(stream_);
  return dtype == SLDM_F32
             ? pool_fwd_t<float>(x, ldx, seg_rowptr, member, piece_ptr, num_segments, num_pieces,
                                 feat, mean_out, ld_mean, max_out, ld_max, max_divisor,
                                 max_first_row, psum, pmax, pcnt, parg, stream)
             : pool_fwd_t<uint16_t>(x, ldx, seg_rowptr, member, piece_ptr, num_segments,
                                    num_pieces, feat, mean_out, ld_mean, max_out, ld_max,
                                    max_divisor, max_first_row, psum, pmax, pcnt, parg, stream);
}

extern "C" int sldm_segment_pool_bwd(int dtype, const void* x, int64_t ldx, const int64_t* seg_of,
                                     const int32_t* seg_rowptr, int64_t num_nodes, int64_t feat,
                                     const void* dmean, int64_t ld_dmean, const void* max_out,
                                     int64_t ld_max, const void* dmax, int64_t ld_dmax,
                                     const float* max_divisor, const int32_t* max_first_row,
                                     void* dx, int64_t ld_dx, void* stream_) {
  SLDM_REQUIRE(dtype == SLDM_F32 || dtype == SLDM_BF16, "sldm_segment_pool_bwd: dtype %d", dtype);
  SLDM_REQUIRE(num_nodes >= 0 && feat >= 0 && feat <= 4096, "sldm_segment_pool_bwd: bad sizes");
  if (num_nodes == 0 || feat == 0) return SLDM_OK;
  SLDM_REQUIRE(seg_of && seg_rowptr && dx && ld_dx >= feat, "sldm_segment_pool_bwd: bad output");
  SLDM_REQUIRE(dmean || dmax, "sldm_segment_pool_bwd: no upstream gradient");
  SLDM_REQUIRE(!dmax || max_first_row || (x && max_out && max_divisor && ldx >= feat),
               "sldm_segment_pool_bwd: the max branch needs the first-max rows, or x, the max "
               "and its divisor");
  hipStream_t stream = sldm::as_stream(stream_);
  return dtype == SLDM_F32
             ? pool_bwd_t<float>(x, ldx, seg_of, seg_rowptr, num_nodes, feat, dmean, ld_dmean,
                                 max_out, ld_max, dmax, ld_dmax, max_divisor, max_first_row, dx,
                                 ld_dx, stream)
             : pool_bwd_t<uint16_t>(x, ldx, seg_of, seg_rowptr, num_nodes, feat, dmean, ld_dmean,
                                    max_out, ld_max, dmax, ld_dmax, max_divisor, max_first_row,
                                    dx, ld_dx, stream);
}
