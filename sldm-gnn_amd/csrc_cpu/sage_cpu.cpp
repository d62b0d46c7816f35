// Host (CPU) kernels of the SageBlock path for the reference's CPU mode
// (DEVICE = 'cpu', /root/reference/main.py:58; test.py:18): the same
// algorithm as the gfx950 library -- CSR by destination built once, rows
// summed straight from the source rows (no [E, F] message tensor), the
// LayerNorm / activation / dropout stage fused per row, the backward on the
// transpose CSR -- in C++ with OpenMP over rows.  fp32 only (the reference's
// dtype).  Dropout uses the GPU kernels' counter hash (common.hpp), so a CPU
// and a GPU run with the same seed draw the same mask.  The GEMMs of the
// layer are plain library GEMMs (torch.mm on the caller side).
//
// This is a separate library (libsldm_sage_cpu.so, g++ -fopenmp) used only
// for CPU tensors; CUDA tensors always go to libsldm_sage.so, and the GPU
// path has no CPU fallback.
#include "sldm_sage_cpu.h"

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

namespace {

inline uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
inline uint32_t dropout_row_key(uint64_t seed, uint64_t row) {
  return hash32((uint32_t)seed ^ hash32((uint32_t)(seed >> 32) ^ hash32((uint32_t)row) ^
                                        (uint32_t)(row >> 32) * 0x9E3779B9u));
}
inline uint32_t dropout_threshold(float p) {
  return p >= 1.f ? 65536u : (p <= 0.f ? 0u : (uint32_t)(p * 65536.f + 0.5f));
}
inline bool dropout_keep(uint32_t row_key, uint32_t col, uint32_t thr) {
  const uint32_t h = hash32(row_key + (col >> 1) * 0x9E3779B9u);
  return ((col & 1u) ? (h >> 16) : (h & 0xFFFFu)) >= thr;
}
inline float drop_scale(float p) { return p >= 1.f ? 0.f : (p > 0.f ? 1.f / (1.f - p) : 1.f); }

}  // namespace

extern "C" {

// CSR by destination (rowptr, col = sources) and by source (t_rowptr,
// t_col = destinations), each row in original edge order (stable counting
// sort).  Returns 1 if an id is outside [0, N), else 0.  An edge (N, N) is
// padding and is skipped, as in the GPU build.
int sldm_cpu_csr_build(const int64_t* ei, int64_t E, int64_t N, int32_t* rowptr, int32_t* col,
                       int32_t* t_rowptr, int32_t* t_col) {
  const int64_t* src = ei;
  const int64_t* dst = ei + E;
  for (int64_t e = 0; e < E; ++e) {
    if (src[e] == N && dst[e] == N) continue;
    if (src[e] < 0 || src[e] >= N || dst[e] < 0 || dst[e] >= N) return 1;
  }
  auto build = [&](const int64_t* key, const int64_t* val, int32_t* ptr, int32_t* out) {
    std::fill(ptr, ptr + N + 1, 0);
    for (int64_t e = 0; e < E; ++e)
      if (key[e] < N) ptr[key[e] + 1]++;
    for (int64_t i = 0; i < N; ++i) ptr[i + 1] += ptr[i];
    std::vector<int32_t> pos(ptr, ptr + N);
    for (int64_t e = 0; e < E; ++e)
      if (key[e] < N) out[pos[key[e]]++] = (int32_t)val[e];
  };
  build(dst, src, rowptr, col);
  if (t_rowptr) build(src, dst, t_rowptr, t_col);
  return 0;
}

// out[i] = (addend[i] +) sum_{k in row i} x[col[k]]  (/ max(1, deg) if mean);
// fp32 sums in CSR order (the reference's scatter_add_ order).
void sldm_cpu_gather_rows(const float* x, int64_t ldx, const int32_t* rowptr, const int32_t* col,
                          int64_t nrows, int64_t feat, int mean, const float* addend,
                          int64_t lda, float* out, int64_t ldo) {
#pragma omp parallel
  {
    std::vector<float> acc(feat);
#pragma omp for schedule(dynamic, 256)
    for (int64_t i = 0; i < nrows; ++i) {
      std::fill(acc.begin(), acc.end(), 0.f);
      const int beg = rowptr[i], end = rowptr[i + 1];
      for (int k = beg; k < end; ++k) {
        const float* xr = x + (int64_t)col[k] * ldx;
#pragma omp simd
        for (int64_t f = 0; f < feat; ++f) acc[f] += xr[f];
      }
      float* o = out + i * ldo;
      const float cnt = (float)(end - beg > 0 ? end - beg : 1);
      for (int64_t f = 0; f < feat; ++f) {
        float v = mean ? acc[f] / cnt : acc[f];
        o[f] = addend ? addend[i * lda + f] + v : v;
      }
    }
  }
}

// g[i] /= max(1, deg_i) in place (the mean's backward, before the transpose sum)
void sldm_cpu_scale_rows_by_inv_deg(float* d, int64_t ld, const int32_t* rowptr, int64_t nrows,
                                    int64_t feat) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < nrows; ++i) {
    const int deg = rowptr[i + 1] - rowptr[i];
    const float cnt = (float)(deg > 0 ? deg : 1);
    for (int64_t f = 0; f < feat; ++f) d[i * ld + f] = d[i * ld + f] / cnt;
  }
}

// h (+ bias) -> LayerNorm -> (Leaky)ReLU -> dropout, per row; saves xhat, rstd.
void sldm_cpu_post_fwd(const float* h, int64_t ldh, int64_t nrows, int64_t feat,
                       const float* bias, const float* gamma, const float* beta, float eps,
                       float slope, float drop_p, uint64_t seed, int64_t row_off, float* out,
                       float* xhat, float* rstd) {
  const uint32_t thr = dropout_threshold(drop_p);
  const float sc = drop_scale(drop_p);
  const float inv_f = 1.0f / (float)feat;
#pragma omp parallel
  {
    std::vector<float> v(feat);
#pragma omp for schedule(static)
    for (int64_t i = 0; i < nrows; ++i) {
      float sum = 0.f;
      for (int64_t f = 0; f < feat; ++f) {
        v[f] = h[i * ldh + f] + (bias ? bias[f] : 0.f);
        sum += v[f];
      }
      const float mean = sum * inv_f;
      float sq = 0.f;
      for (int64_t f = 0; f < feat; ++f) {
        const float d = v[f] - mean;
        sq += d * d;
      }
      const float rs = 1.0f / sqrtf(sq * inv_f + eps);
      if (rstd) rstd[i] = rs;
      const uint32_t rkey = dropout_row_key(seed, (uint64_t)(i + row_off));
      for (int64_t f = 0; f < feat; ++f) {
        const float xh = (v[f] - mean) * rs;
        const float y = fmaf(xh, gamma[f], beta[f]);
        const float a = y > 0.f ? y : y * slope;
        const bool keep = drop_p <= 0.f || dropout_keep(rkey, (uint32_t)f, thr);
        out[i * feat + f] = keep ? a * sc : 0.f;
        if (xhat) xhat[i * feat + f] = xh;
      }
    }
  }
}

// Backward of sldm_cpu_post_fwd: dh and the column sums dgamma, dbeta,
// dbias (= sum of dh), each reduced in a fixed order (per-thread blocks of
// rows, then the blocks in order) -- deterministic for a given thread count.
void sldm_cpu_post_bwd(const float* dout, const float* xhat, const float* rstd, int64_t nrows,
                       int64_t feat, const float* gamma, const float* beta, float slope,
                       float drop_p, uint64_t seed, int64_t row_off, float* dh, float* dgamma,
                       float* dbeta, float* dbias) {
  const uint32_t thr = dropout_threshold(drop_p);
  const float sc = drop_scale(drop_p);
  const float inv_f = 1.0f / (float)feat;
  const int64_t nblk = 64;
  std::vector<float> part((size_t)nblk * 3 * feat, 0.f);
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nblk; ++b) {
    std::vector<float> dy(feat), gx(feat);
    float* pg = part.data() + (size_t)b * 3 * feat;
    const int64_t r0 = nrows * b / nblk, r1 = nrows * (b + 1) / nblk;
    for (int64_t i = r0; i < r1; ++i) {
      const uint32_t rkey = dropout_row_key(seed, (uint64_t)(i + row_off));
      const float* xh = xhat + i * feat;
      float s1 = 0.f, s2 = 0.f;
      for (int64_t f = 0; f < feat; ++f) {
        const bool keep = drop_p <= 0.f || dropout_keep(rkey, (uint32_t)f, thr);
        float d = keep ? dout[i * feat + f] * sc : 0.f;
        d = fmaf(xh[f], gamma[f], beta[f]) > 0.f ? d : d * slope;
        dy[f] = d;
        gx[f] = d * gamma[f];
        s1 += gx[f];
        s2 = fmaf(gx[f], xh[f], s2);
      }
      const float m1 = s1 * inv_f, m2 = s2 * inv_f, rs = rstd[i];
      for (int64_t f = 0; f < feat; ++f) {
        const float o = rs * fmaf(-xh[f], m2, gx[f] - m1);
        dh[i * feat + f] = o;
        pg[f] = fmaf(dy[f], xh[f], pg[f]);
        pg[feat + f] += dy[f];
        pg[2 * feat + f] += o;
      }
    }
  }
  for (int64_t f = 0; f < feat; ++f) {
    float a = 0.f, b = 0.f, c = 0.f;
    for (int64_t k = 0; k < nblk; ++k) {
      a += part[(size_t)k * 3 * feat + f];
      b += part[(size_t)k * 3 * feat + feat + f];
      c += part[(size_t)k * 3 * feat + 2 * feat + f];
    }
    dgamma[f] = a;
    dbeta[f] = b;
    dbias[f] = c;
  }
}

// Graph-level readout on the host (grusage.py:119-127, :185): PyG 2.7.0
// global_mean_pool / global_max_pool = utils.scatter(x, batch, reduce) at
// dim_size B.  Rows are visited in order, so a segment's fp32 sum is the
// reference's scatter_add_ order; OpenMP over columns.
void sldm_cpu_segment_pool(const float* x, int64_t ldx, const int64_t* batch, int64_t nrows,
                           int64_t num_segments, int64_t feat, float* mean_out, int64_t ld_mean,
                           float* max_out, int64_t ld_max, float* max_divisor,
                           int32_t* max_first_row) {
  const int64_t B = num_segments;
  std::vector<int64_t> count((size_t)B, 0);
  for (int64_t i = 0; i < nrows; ++i) ++count[(size_t)batch[i]];
#pragma omp parallel for schedule(static)
  for (int64_t f = 0; f < feat; ++f) {
    if (mean_out) {
      for (int64_t b = 0; b < B; ++b) mean_out[b * ld_mean + f] = 0.f;
      for (int64_t i = 0; i < nrows; ++i) mean_out[batch[i] * ld_mean + f] += x[i * ldx + f];
      for (int64_t b = 0; b < B; ++b)
        mean_out[b * ld_mean + f] /= (float)(count[(size_t)b] > 0 ? count[(size_t)b] : 1);
    }
    if (max_out) {
      std::vector<char> seen((size_t)B, 0);
      std::vector<int32_t> ties((size_t)B, 0), first((size_t)B, 0);
      for (int64_t b = 0; b < B; ++b) max_out[b * ld_max + f] = 0.f;   // empty segments
      for (int64_t i = 0; i < nrows; ++i) {
        const int64_t b = batch[i];
        const float v = x[i * ldx + f];
        float& m = max_out[b * ld_max + f];
        if (!seen[(size_t)b] || v > m) {
          m = v;
          seen[(size_t)b] = 1;
          ties[(size_t)b] = 1;
          first[(size_t)b] = (int32_t)i;
        } else if (v == m) {
          ++ties[(size_t)b];
        }
      }
      for (int64_t b = 0; b < B; ++b) {
        // torch's amax backward divides by the entries equal to the result,
        // the zero-initialised output included when the result is 0
        if (max_divisor)
          max_divisor[b * feat + f] =
              (float)(ties[(size_t)b] + (max_out[b * ld_max + f] == 0.f ? 1 : 0));
        if (max_first_row) max_first_row[b * feat + f] = first[(size_t)b];
      }
    }
  }
}

// dx[i] = dmean[b] / count_b + (x[i] == max[b] ? dmax[b] / max_divisor[b] : 0);
// with max_first_row the max term goes to that row alone (x.max(dim)).
void sldm_cpu_segment_pool_bwd(const float* x, int64_t ldx, const int64_t* batch, int64_t nrows,
                               int64_t num_segments, int64_t feat, const float* dmean,
                               int64_t ld_dmean, const float* max_out, int64_t ld_max,
                               const float* dmax, int64_t ld_dmax, const float* max_divisor,
                               const int32_t* max_first_row, float* dx, int64_t ld_dx) {
  std::vector<int64_t> count((size_t)num_segments, 0);
  for (int64_t i = 0; i < nrows; ++i) ++count[(size_t)batch[i]];
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < nrows; ++i) {
    const int64_t b = batch[i];
    const float cnt = (float)(count[(size_t)b] > 0 ? count[(size_t)b] : 1);
    for (int64_t f = 0; f < feat; ++f) {
      float g = dmean ? dmean[b * ld_dmean + f] / cnt : 0.f;
      if (dmax) {
        if (max_first_row) {
          if (max_first_row[b * feat + f] == (int32_t)i) g += dmax[b * ld_dmax + f];
        } else if (x[i * ldx + f] == max_out[b * ld_max + f]) {
          g += dmax[b * ld_dmax + f] / max_divisor[b * feat + f];
        }
      }
      dx[i * ld_dx + f] = g;
    }
  }
}

int sldm_cpu_abi_version(void) { return 2; }

}  // extern "C"
