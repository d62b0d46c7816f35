// Fused layer boundary of the SageBlock backward: the transpose gather of
// layer l (its input gradient) straight into the LayerNorm / activation /
// dropout backward of layer l-1.
//
// Unfused, a boundary is
//   dx_l[i]  = dx_root_l[i] + sum_{k in out(i)} g_l[t_col[k]]     gather_rows (transpose CSR)
//   dh_{l-1} = post_bwd(dout = dx_l, xhat_{l-1}, rstd_{l-1}, ...)  post_bwd_kernel
// and dx_l makes a round trip through HBM (written by the gather, read back
// by post_bwd: 2 N F s bytes).  Here one row group (LPR lanes, V elements
// each) sums row i's gradient in CSR order exactly as gather_rows does,
// rounds it to the storage type (so the result is bit-identical to the
// unfused pair), and applies the post backward to the row it holds:
//   dy = dout * mask * scale, dy *= (y > 0 ? 1 : slope), y = fma(xhat, g, b)
//   gx = dy * g;  dh = rstd * (gx - mean(gx) - xhat * mean(gx * xhat))
// writing dh_{l-1} and accumulating the dgamma / dbeta / dbias column sums
// of layer l-1 in registers.  Grid-stride over rows (row order from the
// optional longest-first schedule), so the column partials stay one per
// block, reduced in LDS and summed by sldm_colsum in a fixed order
// (deterministic), as in post.hip.
//
// Algorithmic bytes: E (4 + F s) + (N+1) 4 + N F s (addend) + N F s (xhat)
// + 4N (rstd) + N F s (dh).
#include "common.hpp"

namespace {

constexpr int kBlock = 256;

// Column partials of dgamma / dbeta / dbias accumulate in place in LDS, one
// row of 3 F floats per row group.  (Keeping them in registers -- a lane's
// columns are fixed -- measured slower at C4, 14.0 vs 13.6 ms: +10 VGPRs take
// the kernel from 4 to 3 waves per SIMD, and the random-row gather needs the
// occupancy more than the LDS traffic costs.)

template <typename T, int V, int NCH, int NT>
__global__ __launch_bounds__(kBlock) void gather_post_bwd_kernel(
    const T* __restrict__ g, int64_t ldg, const int32_t* __restrict__ t_rowptr,
    const int32_t* __restrict__ t_col, const int32_t* __restrict__ order,
    const T* __restrict__ addend, int64_t lda, int64_t nrows, int feat, int lpr_log2,
    const T* __restrict__ xhat, const float* __restrict__ rstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, float slope, float drop_p, float drop_scale, sldm::Seed seed,
    int64_t row_off, T* __restrict__ dh, float* __restrict__ partials) {
  // Contraction off, as in post_bwd_kernel: the same explicit fmas, every
  // other product and sum rounded on its own -> bit-identical dh.
#pragma clang fp contract(off)
  // LDS: this block's column partials [groups][3][feat], accumulated in place
  // (a group's lanes own distinct columns), then gamma | beta [2][feat]:
  // neither lives in registers across the row loop (occupancy).
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int lpr = 1 << lpr_log2;
  const int lane_in_row = threadIdx.x & (lpr - 1);
  const int group = threadIdx.x >> lpr_log2;
  const int groups_per_block = kBlock >> lpr_log2;
  float* gb = red + (size_t)groups_per_block * 3 * feat;
  for (int j = threadIdx.x; j < groups_per_block * 3 * feat; j += kBlock) red[j] = 0.f;
  for (int j = threadIdx.x; j < feat; j += kBlock) {
    gb[j] = gamma[j];
    gb[feat + j] = beta[j];
  }
  __syncthreads();
  float* mine = red + (size_t)group * 3 * feat;

  int f0[NCH];
  bool act[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int f = (lane_in_row + c * lpr) * V;
    act[c] = f < feat;
    f0[c] = act[c] ? f : feat - V;
  }
  const float inv_f = 1.0f / (float)feat;
  const uint32_t dthr = sldm::dropout_threshold(drop_p);
  const int64_t stride = (int64_t)gridDim.x * groups_per_block;
  const int64_t nrounds = (nrows + stride - 1) / stride;

  // row of iteration `it` and its CSR range, one iteration ahead: the next
  // row's rowptr loads are in flight while this row is gathered
  auto row_of = [&](int64_t it, bool& live) -> int64_t {
    const int64_t slot = it * stride + (int64_t)blockIdx.x * groups_per_block + group;
    live = slot < nrows;
    const int64_t s = live ? slot : 0;
    return order ? (int64_t)order[s] : s;
  };
  bool live_n;
  int64_t row_n = row_of(0, live_n);
  int beg_n = t_rowptr[row_n], end_n = t_rowptr[row_n + 1];
  for (int64_t it = 0; it < nrounds; ++it) {
    const bool live = live_n;
    const int64_t row = row_n;
    const int beg = beg_n, end = end_n;
    if (it + 1 < nrounds) {
      row_n = row_of(it + 1, live_n);
      beg_n = t_rowptr[row_n];
      end_n = t_rowptr[row_n + 1];
    }

    // xhat / rstd / addend of the row first: in flight beside the gather
    float xh[NCH][V], ad[NCH][V];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      sldm::load_vec<T, V, sldm::kStreamOperandsNt && (NT & 1) != 0>(
          xhat + row * (int64_t)feat + f0[c], xh[c]);
      sldm::load_vec<T, V, sldm::kStreamOperandsNt && (NT & 1) != 0>(addend + row * lda + f0[c],
                                                                      ad[c]);
    }
    const float rs = rstd[row];

    // ---- transpose gather of row `row` (gather.hip's batching, CSR order)
    float acc[NCH][V];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[c][v] = 0.f;
    auto batch = [&](int k, auto u_const) {
      constexpr int U = decltype(u_const)::value;
      int idx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) idx[u] = t_col[k + u];
      float d[U][NCH][V];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < NCH; ++c)
          sldm::load_vec<T, V, (NT & 2) != 0>(g + (int64_t)idx[u] * ldg + f0[c], d[u][c]);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int v = 0; v < V; ++v) acc[c][v] += d[u][c][v];
    };
    int k = beg;
    for (; k + 8 <= end; k += 8) batch(k, std::integral_constant<int, 8>{});
    if (k + 4 <= end) { batch(k, std::integral_constant<int, 4>{}); k += 4; }
    if (k + 2 <= end) { batch(k, std::integral_constant<int, 2>{}); k += 2; }
    if (k < end) batch(k, std::integral_constant<int, 1>{});
    float go[NCH][V];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int v = 0; v < V; ++v) go[c][v] = sldm::stored_value<T>(ad[c][v] + acc[c][v]);
    }

    // ---- post backward of the layer below on that row (post.hip's math)
    const float* gbr = gb;
    asm volatile("" : "+v"(gbr));   // per-row LDS reads, not loop-invariant registers
    const uint32_t rkey = sldm::dropout_row_key(sldm::effective_seed(seed), (uint64_t)(row + row_off));
    float gx[NCH][V], dy[NCH][V];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      bool kp[V];
#pragma unroll
      for (int v = 0; v < V; ++v) kp[v] = true;
      if (drop_p > 0.f) sldm::dropout_keepv<V>(rkey, (uint32_t)f0[c], dthr, kp);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float gm = gbr[f0[c] + v], bt = gbr[feat + f0[c] + v];
        float d = kp[v] ? go[c][v] * drop_scale : 0.f;
        d = __builtin_fmaf(xh[c][v], gm, bt) > 0.f ? d : d * slope;
        if (!act[c] || !live) { d = 0.f; xh[c][v] = 0.f; }
        dy[c][v] = d;
        gx[c][v] = d * gm;
        s1 += gx[c][v];
        s2 = __builtin_fmaf(gx[c][v], xh[c][v], s2);
      }
    }
    const float m1 = sldm::group_sum(s1, lpr) * inv_f;
    const float m2 = sldm::group_sum(s2, lpr) * inv_f;
    if (!live) continue;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (!act[c]) continue;
      float o[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        o[v] = rs * __builtin_fmaf(-xh[c][v], m2, gx[c][v] - m1);
        mine[f0[c] + v] = __builtin_fmaf(dy[c][v], xh[c][v], mine[f0[c] + v]);
        mine[feat + f0[c] + v] += dy[c][v];
        mine[2 * feat + f0[c] + v] += o[v];
      }
      sldm::store_vec<T, V, (NT & 1) != 0>(dh + row * (int64_t)feat + f0[c], o);
    }
  }

  __syncthreads();
  for (int j = threadIdx.x; j < 3 * feat; j += kBlock) {
    float acc = 0.f;
    for (int gi = 0; gi < groups_per_block; ++gi) acc += red[(size_t)gi * 3 * feat + j];
    partials[(size_t)blockIdx.x * 3 * feat + j] = acc;
  }
}

template <typename T, int V>
int launch_v(int nch, int lpr_log2, int np, const void* g, int64_t ldg, const int32_t* t_rowptr,
             const int32_t* t_col, const int32_t* order, const void* addend, int64_t lda,
             int64_t nrows, int feat, const void* xhat, const float* rstd, const float* gamma,
             const float* beta, float slope, float p, float scale, uint64_t seed, int64_t row_off,
             void* dh, float* partials, hipStream_t stream) {
  const size_t lds = sizeof(float) * (size_t)feat * (3 * (kBlock >> lpr_log2) + 2);
  SLDM_REQUIRE(lds <= 160 * 1024, "sldm_gather_post_bwd: feat=%d needs %zu B of LDS", feat, lds);
  // non-temporal dh stores on GiB-scale tables (common.hpp nt_gather)
  const int nt = sldm::nt_gather(nrows * ldg * (int64_t)sizeof(T));
#define SLDM_GPB_LAUNCH(NC, NTV)                                                               \
  gather_post_bwd_kernel<T, V, NC, NTV><<<np, kBlock, lds, stream>>>(                          \
      (const T*)g, ldg, t_rowptr, t_col, order, (const T*)addend, lda, nrows, feat,            \
      lpr_log2, (const T*)xhat, rstd, gamma, beta, slope, p, scale, seed, row_off, (T*)dh,     \
      partials)
#define SLDM_GPB_CASE(NC)                                                                      \
  case NC:                                                                                     \
    if (nt == 3) SLDM_GPB_LAUNCH(NC, 3);                                                       \
    else if (nt == 1) SLDM_GPB_LAUNCH(NC, 1);                                                  \
    else SLDM_GPB_LAUNCH(NC, 0);                                                               \
    break;
  switch (nch) {
    SLDM_GPB_CASE(1)
    SLDM_GPB_CASE(2)
    SLDM_GPB_CASE(4)
    default:
      sldm::set_error("sldm_gather_post_bwd: feat=%d unsupported (chunks %d)", feat, nch);
      return SLDM_ERR_ARG;
  }
#undef SLDM_GPB_CASE
#undef SLDM_GPB_LAUNCH
  SLDM_LAUNCH_CHECK("gather_post_bwd_kernel");
  return SLDM_OK;
}

}  // namespace

extern "C" int sldm_gather_post_bwd_num_partials(int64_t num_rows, int64_t feat) {
  if (num_rows <= 0 || feat <= 0) return 1;
  const int lpr = sldm::lanes_per_row(feat, 4);
  const int64_t groups = kBlock / lpr;
  int64_t np = (num_rows + groups * 4 - 1) / (groups * 4);   // >= 4 rows per group
  return (int)(np < 1 ? 1 : (np > 2048 ? 2048 : np));
}

extern "C" int sldm_gather_post_bwd(int dtype, const void* g, int64_t ldg,
                                    const int32_t* t_rowptr, const int32_t* t_col,
                                    const int32_t* row_order, const void* addend, int64_t lda,
                                    int64_t num_rows, int64_t feat, const void* xhat,
                                    const float* rstd, const float* gamma, const float* beta,
                                    float negative_slope, float drop_p, uint64_t seed,
                                    int64_t row_off, void* dh, float* col_partials,
                                    int num_partials, void* stream_) {
  SLDM_REQUIRE(dtype == SLDM_F32 || dtype == SLDM_BF16, "sldm_gather_post_bwd: dtype %d", dtype);
  SLDM_REQUIRE(feat > 0 && feat <= 4096 && num_rows >= 0, "sldm_gather_post_bwd: bad sizes");
  SLDM_REQUIRE(num_partials >= 1 && num_partials <= 4096,
               "sldm_gather_post_bwd: num_partials=%d", num_partials);
  SLDM_REQUIRE(g && t_rowptr && t_col && addend && xhat && rstd && gamma && beta && dh &&
                   col_partials,
               "sldm_gather_post_bwd: NULL argument");
  SLDM_REQUIRE(ldg >= feat && lda >= feat, "sldm_gather_post_bwd: leading dimension < feat");
  SLDM_REQUIRE(drop_p >= 0.0f && drop_p <= 1.0f, "sldm_gather_post_bwd: drop_p=%g",
               (double)drop_p);
  const float scale = drop_p >= 1.0f ? 0.0f : (drop_p > 0.0f ? 1.0f / (1.0f - drop_p) : 1.0f);
  hipStream_t stream = sldm::as_stream(stream_);
  const int eb = dtype == SLDM_F32 ? 4 : 2;
  const int v = sldm::pick_vec(eb, feat, {ldg, lda, feat}, {g, addend, xhat, dh});
  const int lpr = sldm::lanes_per_row(feat, v);
  int lpr_log2 = 0;
  while ((1 << lpr_log2) < lpr) ++lpr_log2;
  const int nch = (int)((feat + (int64_t)lpr * v - 1) / ((int64_t)lpr * v));
  const int f = (int)feat;
#define SLDM_GPB_ARGS                                                                        \
  nch, lpr_log2, num_partials, g, ldg, t_rowptr, t_col, row_order, addend, lda, num_rows, f, \
      xhat, rstd, gamma, beta, negative_slope, drop_p, scale, seed, row_off, dh, col_partials, \
      stream
  if (dtype == SLDM_BF16) {
    switch (v) {
      case 8: return launch_v<uint16_t, 8>(SLDM_GPB_ARGS);
      case 4: return launch_v<uint16_t, 4>(SLDM_GPB_ARGS);
      case 2: return launch_v<uint16_t, 2>(SLDM_GPB_ARGS);
      default: return launch_v<uint16_t, 1>(SLDM_GPB_ARGS);
    }
  }
  switch (v) {
    case 4: return launch_v<float, 4>(SLDM_GPB_ARGS);
    case 2: return launch_v<float, 2>(SLDM_GPB_ARGS);
    default: return launch_v<float, 1>(SLDM_GPB_ARGS);
  }
#undef SLDM_GPB_ARGS
}
