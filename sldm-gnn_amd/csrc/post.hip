// Post-conv elementwise stage of a SageBlock layer:
// lin_l bias -> LayerNorm(F_out, eps) -> LeakyReLU(ns)/ReLU -> Dropout(p),
// /root/reference/src/models/blocks/sageblock.py:9-15, and its backward.
//
// Row-wise and HBM-bound: a row is owned by LPR lanes (power of two <= 64),
// each holding NCH x V consecutive features in registers, so the LayerNorm
// statistics need only lane shuffles (two-pass mean / variance in fp32).
// Dropout uses a counter-based hash of (seed, row*F + col) so the backward
// regenerates the mask instead of storing it.
#include "common.hpp"

namespace {

constexpr int kBlock = 256;

using sldm::group_sum;

template <typename TH, typename TO, int V, int NCH>
__global__ __launch_bounds__(kBlock) void post_fwd_kernel(
    const TH* __restrict__ h, int64_t ldh, int64_t nrows, int feat, int lpr_log2,
    const float* __restrict__ bias, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float slope, float drop_p, float drop_scale,
    sldm::Seed seed, int64_t row_off, TO* __restrict__ out, TO* __restrict__ xhat_out, float* __restrict__ rstd_out) {
  const int lpr = 1 << lpr_log2;
  const int lane_in_row = threadIdx.x & (lpr - 1);
  const int64_t row = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lpr_log2;
  const bool live = row < nrows;  // dead lanes still take part in the shuffles
  const int64_t r = live ? row : 0;

  int f0[NCH];
  bool act[NCH];
  float v[NCH][V];
  float sum = 0.0f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    int f = (lane_in_row + c * lpr) * V;
    act[c] = f < feat;
    f0[c] = act[c] ? f : feat - V;
    sldm::Vec<TH, V>::load(h + r * ldh + f0[c], v[c]);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if (bias) v[c][k] += bias[f0[c] + k];
      if (!act[c]) v[c][k] = 0.0f;
      sum += v[c][k];
    }
  }
  const float inv_f = 1.0f / (float)feat;
  const float mean = group_sum(sum, lpr) * inv_f;
  float sq = 0.0f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float dlt = act[c] ? v[c][k] - mean : 0.0f;
      sq += dlt * dlt;
    }
  const float var = group_sum(sq, lpr) * inv_f;
  const float rstd = 1.0f / sqrtf(var + eps);
  if (!live) return;
  if (rstd_out && lane_in_row == 0) rstd_out[row] = rstd;
  const uint32_t rkey = sldm::dropout_row_key(sldm::effective_seed(seed), (uint64_t)(row + row_off));
  const uint32_t dthr = sldm::dropout_threshold(drop_p);

#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (!act[c]) continue;
    float xh[V], z[V];
    bool keep[V];
#pragma unroll
    for (int k = 0; k < V; ++k) keep[k] = true;
    if (drop_p > 0.0f) sldm::dropout_keepv<V>(rkey, (uint32_t)f0[c], dthr, keep);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int f = f0[c] + k;
      xh[k] = (v[c][k] - mean) * rstd;
      float y = __builtin_fmaf(xh[k], gamma[f], beta[f]);   // the backward recomputes this
      float a = y > 0.0f ? y : y * slope;
      z[k] = keep[k] ? a * drop_scale : 0.0f;
    }
    sldm::Vec<TO, V>::store(out + row * (int64_t)feat + f0[c], z);
    if (xhat_out) sldm::Vec<TO, V>::store(xhat_out + row * (int64_t)feat + f0[c], xh);
  }
}

// One block per partial; grid-stride over row groups.  Column partials are
// kept per thread (fixed columns), then combined across the block's row
// groups in LDS and written as partials[blockIdx.x][3][feat].
// ZOUT (the saved-output branch source) is a template parameter: as a runtime
// test its conditional load put a branch between the row loads, and the
// compiler's vmcnt bookkeeping then drained every row's loads (vmcnt(0))
// before issuing the next row's.  With both rows in flight the C4 time is the
// same (3.26-3.30 ms; selects instead of the per-element branches: 3.46-3.50),
// against 2.52 ms for torch.add over the same 2R:1W bytes: the loop's VALU
// (LN math, dropout hash, exec-mask bookkeeping) is what holds it at
// ~4.7 TB/s, not memory-level parallelism.
template <typename T, typename TD, int V, int NCH, bool ZOUT>
__global__ __launch_bounds__(kBlock) void post_bwd_kernel(
    const T* __restrict__ dout, const T* __restrict__ xhat, const T* __restrict__ zout,
    const float* __restrict__ rstd,
    int64_t nrows, int feat, int lpr_log2, const float* __restrict__ gamma,
    const float* __restrict__ beta, float slope, float drop_p, float drop_scale, sldm::Seed seed, int64_t row_off,
    TD* __restrict__ dh, float* __restrict__ partials) {
  // Contraction off: every product rounds on its own and the fmas are the
  // explicit ones, so gather_post.hip's fused copy of this math gives the
  // same bits whatever the compiler fuses in either kernel.
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float red[];  // [kBlock/lpr][3][feat] reused
  const int lpr = 1 << lpr_log2;
  const int lane_in_row = threadIdx.x & (lpr - 1);
  const int group = threadIdx.x >> lpr_log2;
  const int groups_per_block = kBlock >> lpr_log2;

  int f0[NCH];
  bool act[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    int f = (lane_in_row + c * lpr) * V;
    act[c] = f < feat;
    f0[c] = act[c] ? f : feat - V;
  }
  float pg[NCH][V], pb[NCH][V], pd[NCH][V];
  // gamma / beta of this thread's (fixed) columns, once
  float gm[NCH][V], bt[NCH][V];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int k = 0; k < V; ++k) {
      pg[c][k] = pb[c][k] = pd[c][k] = 0.0f;
      gm[c][k] = gamma[f0[c] + k];
      bt[c][k] = beta[f0[c] + k];
    }

  const float inv_f = 1.0f / (float)feat;
  const uint32_t dthr = sldm::dropout_threshold(drop_p);
  // RB rows per thread group and iteration, all loads issued before the
  // first use (bytes in flight: this kernel is HBM-bound)
#ifndef SLDM_POST_RB
#define SLDM_POST_RB 2
#endif
  constexpr int RB = SLDM_POST_RB;
  const int64_t stride = (int64_t)gridDim.x * groups_per_block;
  const int64_t nrounds = (nrows + RB * stride - 1) / (RB * stride);
  for (int64_t it = 0; it < nrounds; ++it) {
    int64_t rr[RB];
    bool live[RB];
    float go[RB][NCH][V], xh[RB][NCH][V], zo[RB][NCH][ZOUT ? V : 1], rsv[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t row = (it * RB + u) * stride + (int64_t)blockIdx.x * groups_per_block + group;
      live[u] = row < nrows;
      rr[u] = live[u] ? row : 0;
      rsv[u] = rstd[rr[u]];   // with the row loads, not after them
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        sldm::Vec<T, V>::load(dout + rr[u] * (int64_t)feat + f0[c], go[u][c]);
        sldm::Vec<T, V>::load(xhat + rr[u] * (int64_t)feat + f0[c], xh[u][c]);
        if constexpr (ZOUT) sldm::Vec<T, V>::load(zout + rr[u] * (int64_t)feat + f0[c], zo[u][c]);
      }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t r = rr[u];
      const float rs = rsv[u];
      const uint32_t rkey = sldm::dropout_row_key(sldm::effective_seed(seed), (uint64_t)(r + row_off));
      float gx[NCH][V], dy[NCH][V];
      float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        bool kp[V];
#pragma unroll
        for (int k = 0; k < V; ++k) kp[k] = true;
        if (drop_p > 0.0f) sldm::dropout_keepv<V>(rkey, (uint32_t)f0[c], dthr, kp);
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const float g = gm[c][k];
          const bool keep = kp[k];
          float d = keep ? go[u][c][k] * drop_scale : 0.0f;
          // Activation branch: from the saved output when given (sign(z) ==
          // sign(y) exactly, even with bf16 storage); else from
          // y = fma(xhat, g, b), the forward epilogues' exact expression
          // (bit-equal y for fp32 storage; a bf16-rounded xhat can flip only
          // |y| within half an ulp of 0).
          bool pos;
          if constexpr (ZOUT) pos = keep ? zo[u][c][k] > 0.0f : true;
          else pos = __builtin_fmaf(xh[u][c][k], g, bt[c][k]) > 0.0f;
          d = pos ? d : d * slope;
          if (!act[c] || !live[u]) { d = 0.0f; xh[u][c][k] = 0.0f; }
          dy[c][k] = d;
          gx[c][k] = d * g;
          s1 += gx[c][k];
          s2 = __builtin_fmaf(gx[c][k], xh[u][c][k], s2);
        }
      }
      const float m1 = group_sum(s1, lpr) * inv_f;
      const float m2 = group_sum(s2, lpr) * inv_f;
      if (!live[u]) continue;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (!act[c]) continue;
        float o[V];
#pragma unroll
        for (int k = 0; k < V; ++k) {
          o[k] = rs * __builtin_fmaf(-xh[u][c][k], m2, gx[c][k] - m1);
          pg[c][k] = __builtin_fmaf(dy[c][k], xh[u][c][k], pg[c][k]);
          pb[c][k] += dy[c][k];
          pd[c][k] += o[k];
        }
        sldm::Vec<TD, V>::store(dh + r * (int64_t)feat + f0[c], o);
      }
    }
  }

  // Block reduction of the column partials: groups_per_block rows of [3][feat].
  float* mine = red + (size_t)group * 3 * feat;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (!act[c]) continue;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      mine[f0[c] + k] = pg[c][k];
      mine[feat + f0[c] + k] = pb[c][k];
      mine[2 * feat + f0[c] + k] = pd[c][k];
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 3 * feat; j += kBlock) {
    float s = 0.0f;
    for (int g = 0; g < groups_per_block; ++g) s += red[(size_t)g * 3 * feat + j];
    partials[(size_t)blockIdx.x * 3 * feat + j] = s;
  }
}

// out[j] = sum_p partials[p][j]: a block owns 32 columns; its 8 row groups sum
// the partials p == g (mod 8) (4 loads in flight each), then one thread adds
// the 8 group sums in order: fixed order, deterministic.
__global__ __launch_bounds__(kBlock) void colsum_kernel(const float* __restrict__ partials,
                                                        int np, int64_t width,
                                                        float* __restrict__ out) {
  __shared__ float acc[8][32];
  const int c = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t j = (int64_t)blockIdx.x * 32 + c;
  const int64_t jj = j < width ? j : width - 1;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int p = g;
  for (; p + 24 < np; p += 32) {
    s0 += partials[(int64_t)p * width + jj];
    s1 += partials[(int64_t)(p + 8) * width + jj];
    s2 += partials[(int64_t)(p + 16) * width + jj];
    s3 += partials[(int64_t)(p + 24) * width + jj];
  }
  for (; p < np; p += 8) s0 += partials[(int64_t)p * width + jj];
  acc[g][c] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && j < width) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += acc[k][c];
    out[j] = s;
  }
}

struct RowGeom {
  int v, lpr, lpr_log2, nch;
};

RowGeom row_geom(int elem_bytes, int64_t feat, std::initializer_list<const void*> ptrs) {
  RowGeom g;
  g.v = sldm::pick_vec(elem_bytes, feat, {feat}, ptrs);
  g.lpr = sldm::lanes_per_row(feat, g.v);
  g.lpr_log2 = 0;
  while ((1 << g.lpr_log2) < g.lpr) ++g.lpr_log2;
  g.nch = (int)((feat + (int64_t)g.lpr * g.v - 1) / ((int64_t)g.lpr * g.v));
  return g;
}

template <typename TH, typename TO, int V>
int post_fwd_nch(const RowGeom& g, const void* h, int64_t ldh, int64_t nrows, int feat,
                 const float* bias, const float* gamma, const float* beta, float eps,
                 float slope, float p, float scale, uint64_t seed, int64_t row_off, void* out, void* xhat,
                 float* rstd, hipStream_t stream) {
  const int64_t grid = ((nrows << g.lpr_log2) + kBlock - 1) / kBlock;
#define SLDM_PF_CASE(NC)                                                                     \
  case NC:                                                                                   \
    post_fwd_kernel<TH, TO, V, NC><<<(unsigned)grid, kBlock, 0, stream>>>(                   \
        reinterpret_cast<const TH*>(h), ldh, nrows, feat, g.lpr_log2, bias, gamma, beta,     \
        eps, slope, p, scale, seed, row_off, reinterpret_cast<TO*>(out), reinterpret_cast<TO*>(xhat), \
        rstd);                                                                               \
    break;
  switch (g.nch) {
    SLDM_PF_CASE(1)
    SLDM_PF_CASE(2)
    SLDM_PF_CASE(4)
    default:
      sldm::set_error("sldm_post_fwd: feat=%d unsupported (chunks %d)", feat, g.nch);
      return SLDM_ERR_ARG;
  }
#undef SLDM_PF_CASE
  SLDM_LAUNCH_CHECK("post_fwd_kernel");
  return SLDM_OK;
}

template <typename T, typename TD, int V>
int post_bwd_nch(const RowGeom& g, const void* dout, const void* xhat, const void* zout, const float* rstd,
                 int64_t nrows, int feat, const float* gamma, const float* beta, float slope,
                 float p, float scale, uint64_t seed, int64_t row_off, void* dh, float* partials, int np,
                 hipStream_t stream) {
  const size_t lds = sizeof(float) * 3 * (size_t)feat * (kBlock >> g.lpr_log2);
  if (lds > 160 * 1024) {
    sldm::set_error("sldm_post_bwd: feat=%d needs %zu B of LDS", feat, lds);
    return SLDM_ERR_ARG;
  }
#define SLDM_PB_CASE(NC)                                                                       \
  case NC:                                                                                     \
    if (zout)                                                                                  \
      post_bwd_kernel<T, TD, V, NC, true><<<np, kBlock, lds, stream>>>(                        \
          reinterpret_cast<const T*>(dout), reinterpret_cast<const T*>(xhat),                  \
          reinterpret_cast<const T*>(zout), rstd, nrows, feat, g.lpr_log2, gamma, beta, slope, \
          p, scale, seed, row_off, reinterpret_cast<TD*>(dh), partials);                       \
    else                                                                                       \
      post_bwd_kernel<T, TD, V, NC, false><<<np, kBlock, lds, stream>>>(                       \
          reinterpret_cast<const T*>(dout), reinterpret_cast<const T*>(xhat), nullptr, rstd,   \
          nrows, feat, g.lpr_log2, gamma, beta, slope, p, scale, seed, row_off,                \
          reinterpret_cast<TD*>(dh), partials);                                                \
    break;
  switch (g.nch) {
    SLDM_PB_CASE(1)
    SLDM_PB_CASE(2)
    SLDM_PB_CASE(4)
    default:
      sldm::set_error("sldm_post_bwd: feat=%d unsupported (chunks %d)", feat, g.nch);
      return SLDM_ERR_ARG;
  }
#undef SLDM_PB_CASE
  SLDM_LAUNCH_CHECK("post_bwd_kernel");
  return SLDM_OK;
}

template <typename TH, typename TO>
int post_fwd_t(const RowGeom& g, const void* h, int64_t ldh, int64_t nrows, int feat,
               const float* bias, const float* gamma, const float* beta, float eps, float slope,
               float p, float scale, uint64_t seed, int64_t row_off, void* out, void* xhat, float* rstd,
               hipStream_t stream) {
  switch (g.v) {
    case 8:
      if constexpr (sizeof(TH) == 2 && sizeof(TO) == 2)
        return post_fwd_nch<TH, TO, 8>(g, h, ldh, nrows, feat, bias, gamma, beta, eps, slope, p, scale, seed, row_off, out, xhat, rstd, stream);
      break;
    case 4:
      return post_fwd_nch<TH, TO, 4>(g, h, ldh, nrows, feat, bias, gamma, beta, eps, slope, p, scale, seed, row_off, out, xhat, rstd, stream);
    case 2:
      return post_fwd_nch<TH, TO, 2>(g, h, ldh, nrows, feat, bias, gamma, beta, eps, slope, p, scale, seed, row_off, out, xhat, rstd, stream);
    case 1:
      return post_fwd_nch<TH, TO, 1>(g, h, ldh, nrows, feat, bias, gamma, beta, eps, slope, p, scale, seed, row_off, out, xhat, rstd, stream);
  }
  sldm::set_error("sldm_post_fwd: vector width %d", g.v);
  return SLDM_ERR_ARG;
}

template <typename T, typename TD>
int post_bwd_t(const RowGeom& g, const void* dout, const void* xhat, const void* zout, const float* rstd,
               int64_t nrows, int feat, const float* gamma, const float* beta, float slope,
               float p, float scale, uint64_t seed, int64_t row_off, void* dh, float* partials, int np,
               hipStream_t stream) {
  switch (g.v) {
    case 8:
      if constexpr (sizeof(T) == 2 && sizeof(TD) == 2)
        return post_bwd_nch<T, TD, 8>(g, dout, xhat, zout, rstd, nrows, feat, gamma, beta, slope, p, scale, seed, row_off, dh, partials, np, stream);
      break;
    case 4:
      return post_bwd_nch<T, TD, 4>(g, dout, xhat, zout, rstd, nrows, feat, gamma, beta, slope, p, scale, seed, row_off, dh, partials, np, stream);
    case 2:
      return post_bwd_nch<T, TD, 2>(g, dout, xhat, zout, rstd, nrows, feat, gamma, beta, slope, p, scale, seed, row_off, dh, partials, np, stream);
    case 1:
      return post_bwd_nch<T, TD, 1>(g, dout, xhat, zout, rstd, nrows, feat, gamma, beta, slope, p, scale, seed, row_off, dh, partials, np, stream);
  }
  sldm::set_error("sldm_post_bwd: vector width %d", g.v);
  return SLDM_ERR_ARG;
}

}  // namespace

extern "C" int sldm_post_fwd(int h_dtype, const void* h, int64_t ldh, int64_t num_rows,
                             int64_t feat, const float* bias, const float* gamma,
                             const float* beta, float eps, float negative_slope, float drop_p,
                             uint64_t seed, int64_t row_off, int out_dtype, void* out, void* xhat, float* rstd,
                             void* stream_) {
  SLDM_REQUIRE(num_rows >= 0 && feat > 0 && feat <= 4096, "sldm_post_fwd: bad sizes");
  if (num_rows == 0) return SLDM_OK;
  SLDM_REQUIRE(h && gamma && beta && out && ldh >= feat, "sldm_post_fwd: bad arguments");
  SLDM_REQUIRE(drop_p >= 0.0f && drop_p <= 1.0f, "sldm_post_fwd: drop_p=%g outside [0,1]",
               (double)drop_p);
  const float scale = drop_p >= 1.0f ? 0.0f : (drop_p > 0.0f ? 1.0f / (1.0f - drop_p) : 1.0f);
  hipStream_t stream = sldm::as_stream(stream_);
  const int f = (int)feat;
  int hb = h_dtype == SLDM_F32 ? 4 : 2, ob = out_dtype == SLDM_F32 ? 4 : 2;
  RowGeom g = row_geom(hb > ob ? ob : hb, feat, {h, out, xhat});
  if (h_dtype == SLDM_F32 || out_dtype == SLDM_F32) {
    // Vector width is shared between input and output: cap it at 4.
    if (g.v > 4) { g = row_geom(4, feat, {h, out, xhat}); }
  }
  SLDM_REQUIRE(ldh % g.v == 0, "sldm_post_fwd: ldh not aligned");
  if (h_dtype == SLDM_F32 && out_dtype == SLDM_F32)
    return post_fwd_t<float, float>(g, h, ldh, num_rows, f, bias, gamma, beta, eps, negative_slope, drop_p, scale, seed, row_off, out, xhat, rstd, stream);
  if (h_dtype == SLDM_BF16 && out_dtype == SLDM_BF16)
    return post_fwd_t<uint16_t, uint16_t>(g, h, ldh, num_rows, f, bias, gamma, beta, eps, negative_slope, drop_p, scale, seed, row_off, out, xhat, rstd, stream);
  if (h_dtype == SLDM_F32 && out_dtype == SLDM_BF16)
    return post_fwd_t<float, uint16_t>(g, h, ldh, num_rows, f, bias, gamma, beta, eps, negative_slope, drop_p, scale, seed, row_off, out, xhat, rstd, stream);
  sldm::set_error("sldm_post_fwd: dtype pair (%d -> %d) unsupported", h_dtype, out_dtype);
  return SLDM_ERR_ARG;
}

extern "C" int sldm_post_num_partials(int64_t num_rows, int64_t feat) {
  if (num_rows <= 0 || feat <= 0) return 1;
  RowGeom g = row_geom(4, feat, {});
  const int64_t groups = kBlock >> g.lpr_log2;
  int64_t np = (num_rows + groups * 4 - 1) / (groups * 4);  // >= 4 rows per group
  if (np > 2048) np = 2048;
  return (int)(np < 1 ? 1 : np);
}

extern "C" int sldm_post_bwd(int dtype, const void* dout, const void* xhat, const void* zout, const float* rstd,
                             int64_t num_rows, int64_t feat, const float* gamma,
                             const float* beta, float negative_slope, float drop_p,
                             uint64_t seed, int64_t row_off, int dh_dtype, void* dh, float* col_partials,
                             int num_partials, void* stream_) {
  SLDM_REQUIRE(feat > 0 && feat <= 4096 && num_rows >= 0, "sldm_post_bwd: bad sizes");
  SLDM_REQUIRE(num_partials >= 1 && num_partials <= 4096, "sldm_post_bwd: num_partials=%d",
               num_partials);
  SLDM_REQUIRE(dout && xhat && rstd && gamma && beta && dh && col_partials,
               "sldm_post_bwd: NULL argument");
  SLDM_REQUIRE(drop_p >= 0.0f && drop_p <= 1.0f, "sldm_post_bwd: drop_p=%g outside [0,1]",
               (double)drop_p);
  const float scale = drop_p >= 1.0f ? 0.0f : (drop_p > 0.0f ? 1.0f / (1.0f - drop_p) : 1.0f);
  hipStream_t stream = sldm::as_stream(stream_);
  const int f = (int)feat;
  int eb = (dtype == SLDM_F32 || dh_dtype == SLDM_F32) ? 4 : 2;
  RowGeom g = row_geom(eb, feat, {dout, xhat, dh});
  if (dtype == SLDM_F32 && dh_dtype == SLDM_F32)
    return post_bwd_t<float, float>(g, dout, xhat, zout, rstd, num_rows, f, gamma, beta, negative_slope, drop_p, scale, seed, row_off, dh, col_partials, num_partials, stream);
  if (dtype == SLDM_BF16 && dh_dtype == SLDM_BF16)
    return post_bwd_t<uint16_t, uint16_t>(g, dout, xhat, zout, rstd, num_rows, f, gamma, beta, negative_slope, drop_p, scale, seed, row_off, dh, col_partials, num_partials, stream);
  if (dtype == SLDM_BF16 && dh_dtype == SLDM_F32)
    return post_bwd_t<uint16_t, float>(g, dout, xhat, zout, rstd, num_rows, f, gamma, beta, negative_slope, drop_p, scale, seed, row_off, dh, col_partials, num_partials, stream);
  sldm::set_error("sldm_post_bwd: dtype pair (%d, dh %d) unsupported", dtype, dh_dtype);
  return SLDM_ERR_ARG;
}

extern "C" int sldm_colsum(const float* partials, int num_partials, int64_t width, float* out,
                           void* stream_) {
  SLDM_REQUIRE(num_partials >= 1 && width >= 0 && partials && out, "sldm_colsum: bad arguments");
  if (width == 0) return SLDM_OK;
  hipStream_t stream = sldm::as_stream(stream_);
  colsum_kernel<<<(unsigned)((width + 31) / 32), kBlock, 0, stream>>>(
      partials, num_partials, width, out);
  SLDM_LAUNCH_CHECK("colsum_kernel");
  return SLDM_OK;
}
