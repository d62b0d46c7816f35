// The dense part of a SageBlock layer on MFMA:
//
//   forward   h = [agg | x] · [W_l | W_r]^T            (PyG SAGEConv lin_l + lin_r)
//             fused epilogue: + b_l, LayerNorm, LeakyReLU/ReLU, dropout (A7)
//   backward  [dAgg | dx_root] = dh · [W_l | W_r]      (lin_l / lin_r input grads)
//             fused epilogue: dAgg / max(1, deg)        (the mean's backward)
//             [dW_l | dW_r] = dh^T · [agg | x]          (weight grads, split-K)
//
// gemm_nt: C[M,Nc] = A[M,K]·B[Nc,K]^T, both operands K-contiguous, loaded as
//   16-byte fragments straight into the MFMA operand registers (B is the
//   tiny weight matrix, L2-resident; A streams from HBM once per block).
//   Block = 4 waves x (16·MT rows), wave w owns column tiles w, w+4, ...;
//   the next k-step's fragments are in flight while the current one feeds
//   the MFMAs.  The accumulator tile is staged through LDS so the epilogue
//   works on whole rows (LayerNorm statistics by wave reductions) and every
//   store is a coalesced row segment.
//   bf16: v_mfma_f32_16x16x32_bf16 (fp32 accumulate);
//   fp32: v_mfma_f32_16x16x4_f32 (exact fp32 fma chain, no TF32 on gfx950).
//
// gemm_tn: C[Mo,Nn] = sum_k A[k,:]^T ⊗ B[k,:]  (k = node index, huge).  Both
//   operands are k-strided, so 32-row tiles are staged through LDS (row-major,
//   coalesced) and read transposed with ds_read_b64_tr_b16 (bf16) or per-lane
//   ds_read_b32 (fp32).  The node range is split across blocks (split-K);
//   blocks of one split sit on one XCD (blockIdx % 8) so the re-read operand
//   panels hit that XCD's L2; fp32 partial slabs are summed in a fixed order.
#include "common.hpp"

namespace {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;

// ------------------------------------------------------------ NT operands --
template <typename T> struct NtOps;

template <> struct NtOps<uint16_t> {
  static constexpr int EPL = 8;   // k elements per lane per step
  static constexpr int KS = 32;   // k per step = 4 lane groups x EPL
  using Frag = s8v;
  __device__ static Frag zero() { return Frag{0, 0, 0, 0, 0, 0, 0, 0}; }
  __device__ static Frag load(const uint16_t* p) { return *reinterpret_cast<const s8v*>(p); }
  __device__ static void set(Frag& f, int j, uint16_t v) { f[j] = (short)v; }
  __device__ static void mma(f4v& acc, const Frag& a, const Frag& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
};

template <> struct NtOps<float> {
  static constexpr int EPL = 4;
  static constexpr int KS = 16;
  using Frag = f4v;
  __device__ static Frag zero() { return Frag{0.f, 0.f, 0.f, 0.f}; }
  __device__ static Frag load(const float* p) { return *reinterpret_cast<const f4v*>(p); }
  __device__ static void set(Frag& f, int j, float v) { f[j] = v; }
  // Lane group q holds k = k0 + 4q + c in component c: four MFMAs cover the
  // 16 k of the step with A and B indexed by the same k.
  __device__ static void mma(f4v& acc, const Frag& a, const Frag& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], acc, 0, 0, 0);
  }
};

enum { EPI_LN = 0, EPI_ROWSCALE = 1 };

template <typename T>
struct NtArgs {
  const T* a0; int64_t lda0; int k0;   // A columns [0, k0)
  const T* a1; int64_t lda1;           // A columns [k0, K)
  int K;
  const T* b; int64_t ldb;             // B [Nc][K]
  int64_t M; int Nc;
  int ct;                              // 16-column tiles per block
  int grid_y;                          // column blocks
  int kce;                             // K chunk staged in LDS (<= 1 KiB of a row)
  T* out; int64_t ldo;
  // EPI_LN
  T* xhat; float* rstd;
  const float* bias; const float* gamma; const float* beta;
  float eps, slope, drop_p, drop_scale; sldm::Seed seed; int64_t row_off;
  // EPI_ROWSCALE (out2: optional destination of the columns >= scale_cols)
  const int32_t* rowptr; int scale_cols;
  T* out2; int64_t ldo2;
};

template <typename T, bool VEC>
__device__ __forceinline__ typename NtOps<T>::Frag nt_load_a(const NtArgs<T>& p, int64_t row,
                                                             int kk) {
  using O = NtOps<T>;
  typename O::Frag f;
  if constexpr (VEC) {
    // K0 and K are multiples of EPL: a fragment never straddles A0/A1 or K.
    const int kc = kk < p.K ? kk : p.K - O::EPL;
    const T* src = kc < p.k0 ? p.a0 + row * p.lda0 + kc : p.a1 + row * p.lda1 + (kc - p.k0);
    f = O::load(src);
    if (kk >= p.K) f = O::zero();
  } else {
#pragma unroll
    for (int j = 0; j < O::EPL; ++j) {
      const int k = kk + j;
      const int kc = k < p.K ? k : p.K - 1;
      T v = kc < p.k0 ? p.a0[row * p.lda0 + kc] : p.a1[row * p.lda1 + (kc - p.k0)];
      O::set(f, j, k < p.K ? v : (T)0);
    }
  }
  return f;
}

template <typename T, bool VEC>
__device__ __forceinline__ typename NtOps<T>::Frag nt_load_b(const NtArgs<T>& p, int col, int kk) {
  using O = NtOps<T>;
  typename O::Frag f;
  if constexpr (VEC) {
    // VEC: K is a multiple of the k-step, so kk < K always: no select on the
    // loaded value (a select right after a load makes hipcc wait vmcnt(0)).
    f = O::load(p.b + (int64_t)col * p.ldb + kk);
  } else {
#pragma unroll
    for (int j = 0; j < O::EPL; ++j) {
      const int k = kk + j;
      const int kc = k < p.K ? k : p.K - 1;
      T v = p.b[(int64_t)col * p.ldb + kc];
      O::set(f, j, k < p.K ? v : (T)0);
    }
  }
  return f;
}

// Row epilogue of an NT tile whose fp32 accumulators sit in LDS [BM][ldc]:
// a wave owns a row; lane holds columns 4*lane .. 4*lane+3 (4 waves per block).
template <typename T, int MODE>
__device__ __forceinline__ void nt_row_epilogue(const NtArgs<T>& p, const float* smem, int ldc,
                                                int64_t m0, int n0, int BM, int wave, int lane) {
  const int bn_valid = min(16 * p.ct, p.Nc - n0);
  // A row per 32 lanes when it has <= 128 columns (two rows per wave step; the
  // 32-lane sums equal the 64-lane ones, whose upper half added zeros), else
  // per 64 lanes.
  const int lpr = bn_valid > 128 ? 64 : 32;
  const int rpi = 64 / lpr;
  const int c0 = 4 * (lane & (lpr - 1));
  const bool lane_on = c0 < bn_valid;
  const bool full4 = (c0 + 3 < bn_valid) && (p.ldo % 4 == 0);
  // The lane's columns are fixed: bias / gamma / beta are loaded once, not per
  // row (per-row loads put three dependent L1 round trips on every row).
  float bi[4] = {0.f, 0.f, 0.f, 0.f}, ga[4] = {0.f, 0.f, 0.f, 0.f}, be[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE == EPI_LN) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = min(c0 + j, bn_valid - 1);
      if (p.bias) bi[j] = p.bias[c];
      ga[j] = p.gamma[c];
      be[j] = p.beta[c];
    }
  }
  for (int rr = wave * rpi + lane / lpr; rr < BM; rr += 4 * rpi) {
    const int64_t row = m0 + rr;
    if (row >= p.M) break;   // uniform per row group (the sums stay inside it)
    float v[4];
    {
      const f4v t4 = *reinterpret_cast<const f4v*>(&smem[rr * ldc + c0]);
      v[0] = t4[0]; v[1] = t4[1]; v[2] = t4[2]; v[3] = t4[3];
    }
    if constexpr (MODE == EPI_LN) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        const bool ok = lane_on && c < bn_valid;
        v[j] = ok ? v[j] + bi[j] : 0.f;
        s += v[j];
      }
      const float inv_n = 1.0f / (float)p.Nc;
      const float mean = sldm::group_sum(s, lpr) * inv_n;
      float sq = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = (lane_on && c0 + j < bn_valid) ? v[j] - mean : 0.f;
        sq += d * d;
      }
      const float rstd = 1.0f / sqrtf(sldm::group_sum(sq, lpr) * inv_n + p.eps);
      if (p.rstd && (lane & (lpr - 1)) == 0) p.rstd[row] = rstd;
      if (!lane_on) continue;
      const uint32_t rkey = sldm::dropout_row_key(sldm::effective_seed(p.seed), (uint64_t)(row + p.row_off));
      float xh[4], z[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = min(c0 + j, bn_valid - 1);
        xh[j] = (v[j] - mean) * rstd;
        const float y = __builtin_fmaf(xh[j], ga[j], be[j]);   // as post_bwd recomputes it
        float a = y > 0.f ? y : y * p.slope;
        if (p.drop_p > 0.f) {
          a = sldm::dropout_keep(rkey, (uint32_t)c, sldm::dropout_threshold(p.drop_p))
                  ? a * p.drop_scale : 0.f;
        }
        z[j] = a;
      }
      T* orow = p.out + row * p.ldo + n0 + c0;
      T* xrow = p.xhat ? p.xhat + row * p.ldo + n0 + c0 : nullptr;
      if (full4) {
        sldm::Vec<T, 4>::store(orow, z);
        if (xrow) sldm::Vec<T, 4>::store(xrow, xh);
      } else {
        for (int j = 0; j < 4 && c0 + j < bn_valid; ++j) {
          sldm::Vec<T, 1>::store(orow + j, &z[j]);
          if (xrow) sldm::Vec<T, 1>::store(xrow + j, &xh[j]);
        }
      }
    } else {
      if (!lane_on) continue;
      if (p.rowptr) {
        const int deg = p.rowptr[row + 1] - p.rowptr[row];
        const float cnt = (float)(deg > 0 ? deg : 1);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n0 + c0 + j < p.scale_cols) v[j] = v[j] / cnt;
      }
      // split output: columns >= scale_cols go to out2 (scale_cols % 4 == 0,
      // so a 4-column group never straddles the split)
      const bool hi = p.out2 && n0 + c0 >= p.scale_cols;
      T* orow = hi ? p.out2 + row * p.ldo2 + (n0 + c0 - p.scale_cols)
                   : p.out + row * p.ldo + n0 + c0;
      if (full4) {
        sldm::Vec<T, 4>::store(orow, v);
      } else {
        for (int j = 0; j < 4 && c0 + j < bn_valid; ++j) sldm::Vec<T, 1>::store(orow + j, &v[j]);
      }
    }
  }
}

// Row tile (16·MT rows) and resident blocks per CU.  fp32 (exact
// v_mfma_f32_16x16x4_f32, 16x slower per FLOP than bf16) is MFMA-bound and
// hides its per-k-step weight-fragment loads (L2) only with more waves in
// flight: 32-row tiles, 4 blocks per CU (C2, F = 128: LN forward 0.188 ->
// 0.155 ms, dX 0.116 -> 0.103 ms; 8 blocks per CU or 16-row tiles are slower
// -- the weights are re-read from L2 once per tile).  bf16 keeps 64-row tiles.
template <typename T> struct NtTile { static constexpr int MT = 4, MINB = 2; };
template <> struct NtTile<float> { static constexpr int MT = 2, MINB = 4; };

template <typename T, int MT, int TPW, bool VEC, int MODE>
__global__ __launch_bounds__(kBlock, NtTile<T>::MINB) void gemm_nt_kernel(NtArgs<T> p) {
  using O = NtOps<T>;
  using Frag = typename O::Frag;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int BM = 16 * MT;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // SGPR: tile tests are scalar
  const int q = lane >> 4, r16 = lane & 15;

  // Block -> (row block, column block).  With several column blocks, those of
  // one row block share blockIdx % 8 (one XCD's L2 under round-robin
  // dispatch) and run back to back, so the A rows are fetched from HBM once.
  int rb, cb;
  if (p.grid_y > 1) {
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    cb = j % p.grid_y;
    rb = (j / p.grid_y) * 8 + xcd;
  } else {
    rb = blockIdx.x;
    cb = 0;
  }
  const int64_t m0 = (int64_t)rb * BM;
  if (m0 >= p.M) return;  // padding blocks of the XCD mapping (whole block)
  const int n0 = cb * 16 * p.ct;

  int bcol[TPW];
  bool tval[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tid = wave + 4 * t;
    tval[t] = tid < p.ct;
    int c = n0 + 16 * tid + r16;
    bcol[t] = c < p.Nc ? c : p.Nc - 1;
  }

  f4v acc[MT][TPW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[m][t] = f4v{0.f, 0.f, 0.f, 0.f};

  // A row block staged through LDS one K-chunk (kce <= 1 KiB per row) at a
  // time: every thread issues all of its 16-B loads before the first wait,
  // so the whole chunk is in flight at once; the four waves then read their
  // fragments with ds_read_b128 (row pitch = 16 B mod 256 B: conflict-free).
  T* lds_a = reinterpret_cast<T*>(smem);
  const int pa = p.kce + 16 / (int)sizeof(T);
  for (int kc0 = 0; kc0 < p.K; kc0 += p.kce) {
    if (kc0 > 0) __syncthreads();
    if constexpr (VEC) {
      // Two passes, one per source (A0 = columns [0,k0), A1 = [k0,K)), so the
      // source pointer is uniform; rows past M are clamped (computed, never
      // stored).  8 vectors in flight per thread per group, no selects.
      constexpr int EPV = O::EPL;   // 16 B per vector
      constexpr int G = 8;
      const int kc1 = min(kc0 + p.kce, p.K);
#pragma unroll
      for (int part = 0; part < 2; ++part) {
        const int lo = part == 0 ? kc0 : max(kc0, p.k0);
        const int hi = part == 0 ? min(kc1, p.k0) : kc1;
        if (lo >= hi) continue;
        const T* base = part == 0 ? p.a0 + lo : p.a1 + (lo - p.k0);
        const int64_t ld = part == 0 ? p.lda0 : p.lda1;
        const int vpr = (hi - lo) / EPV;
        const int nv = BM * vpr;
        for (int v0 = 0; v0 < nv; v0 += G * kBlock) {
          Frag st[G];
#pragma unroll
          for (int i = 0; i < G; ++i) {
            const int v = v0 + threadIdx.x + i * kBlock;
            const int r = v / vpr;
            const int64_t row = min(m0 + min(r, BM - 1), p.M - 1);
            st[i] = O::load(base + row * ld + (v - r * vpr) * EPV);
          }
#pragma unroll
          for (int i = 0; i < G; ++i) {
            const int v = v0 + threadIdx.x + i * kBlock;
            const int r = v / vpr;
            if (v < nv)
              *reinterpret_cast<Frag*>(lds_a + r * pa + (lo - kc0) + (v - r * vpr) * EPV) = st[i];
          }
        }
      }
    } else {
      constexpr int EPV = O::EPL;
      const int vpr = p.kce / EPV;
      const int nv = BM * vpr;
      for (int v = threadIdx.x; v < nv; v += kBlock) {
        const int r = v / vpr;
        const int kk = kc0 + (v - r * vpr) * EPV;
        Frag f = nt_load_a<T, false>(p, min(m0 + r, p.M - 1), kk);
        *reinterpret_cast<Frag*>(lds_a + r * pa + (kk - kc0)) = f;
      }
    }
    __syncthreads();
    // k extent of this chunk rounded up to the k-step (the staged tile is
    // zero-filled past K; the scalar path bounds-checks its B loads).
    const int kend = min(p.kce, (p.K - kc0 + O::KS - 1) / O::KS * O::KS);
    // B (weight) fragments stream from L2 in batches of two k-steps held in
    // two named register sets (ping-pong, no copies): the batch for steps
    // k+2, k+3 is in flight while steps k, k+1 run their MFMAs.
    Frag bx[2][TPW], by[2][TPW];
    // Loads are unconditional (a step past kend re-reads the last valid one)
    // so hipcc can count them and wait with vmcnt(N) instead of vmcnt(0).
    auto load2 = [&](Frag (&bb)[2][TPW], int k) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ks = min(k + s * O::KS, kend - O::KS);
#pragma unroll
        for (int t = 0; t < TPW; ++t)
          bb[s][t] = nt_load_b<T, VEC>(p, bcol[t], kc0 + ks + O::EPL * q);
      }
    };
    auto mma2 = [&](Frag (&bb)[2][TPW], int k) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (k + s * O::KS < kend) {
          Frag a[MT];
#pragma unroll
          for (int m = 0; m < MT; ++m)
            a[m] = *reinterpret_cast<const Frag*>(lds_a + (16 * m + r16) * pa + k + s * O::KS +
                                                  O::EPL * q);
#pragma unroll
          for (int t = 0; t < TPW; ++t) {
            if (!tval[t]) continue;
#pragma unroll
            for (int m = 0; m < MT; ++m) O::mma(acc[m][t], a[m], bb[s][t]);
          }
        }
      }
    };
    load2(bx, 0);
    for (int k0 = 0; k0 < kend; k0 += 4 * O::KS) {
      load2(by, k0 + 2 * O::KS);
      mma2(bx, k0);
      if (k0 + 2 * O::KS >= kend) break;
      load2(bx, k0 + 4 * O::KS);
      mma2(by, k0 + 2 * O::KS);
    }
  }
  __syncthreads();  // LDS now holds the C tile

  // Accumulator tile -> LDS [BM][ldc] fp32 (C/D map: col = lane&15, row = 4(lane>>4)+r).
  const int ldc = 16 * p.ct + 4;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    if (!tval[t]) continue;
    const int c = 16 * (wave + 4 * t) + r16;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) smem[(16 * m + 4 * q + r) * ldc + c] = acc[m][t][r];
  }
  __syncthreads();

  nt_row_epilogue<T, MODE>(p, smem, ldc, m0, n0, BM, wave, lane);
}

// The fp32 tile kernel with split-bf16 products (fp32 in and out, fp32
// accumulation; K a multiple of 32, 16-B aligned operands).  Each operand
// element is split three ways, x = hi + mid + lo (bf16 each, exact), and a
// product is the six partial products that matter (sldm::split3_bf16x4,
// SLDM_MFMA_X6 in common.hpp): fp32-level results from six 16-cycle
// v_mfma_f32_16x16x32_bf16 per 32-deep k-step against the exact kernel's
// eight 32-cycle 16x16x4 fp32 MFMAs.  The A row block is split while it is
// staged into LDS (three bf16 images); the weight fragments are split in
// registers as they arrive from L2.  Same block / wave / epilogue structure
// as gemm_nt_kernel<float>, on 64-row tiles (the MFMA phase no longer bounds
// the kernel).
template <int MT, int TPW, int MODE>
__global__ __launch_bounds__(kBlock, 2) void gemm_nt_x6_kernel(NtArgs<float> p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int BM = 16 * MT;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, r16 = lane & 15;

  int rb, cb;
  if (p.grid_y > 1) {
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    cb = j % p.grid_y;
    rb = (j / p.grid_y) * 8 + xcd;
  } else {
    rb = blockIdx.x;
    cb = 0;
  }
  const int64_t m0 = (int64_t)rb * BM;
  if (m0 >= p.M) return;
  const int n0 = cb * 16 * p.ct;

  int bcol[TPW];
  bool tval[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tid = wave + 4 * t;
    tval[t] = tid < p.ct;
    int c = n0 + 16 * tid + r16;
    bcol[t] = c < p.Nc ? c : p.Nc - 1;
  }

  f4v acc[MT][TPW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[m][t] = f4v{0.f, 0.f, 0.f, 0.f};

  // hi / mid / lo bf16 images of the staged K chunk: row pitch kce + 8
  // elements (16 B mod 256 B per row pair: conflict-free ds_read_b128)
  const int pa = p.kce + 8;
  uint16_t* img_hi = reinterpret_cast<uint16_t*>(smem);
  uint16_t* img_mid = img_hi + BM * pa;
  uint16_t* img_lo = img_mid + BM * pa;
  for (int kc0 = 0; kc0 < p.K; kc0 += p.kce) {
    if (kc0 > 0) __syncthreads();
    constexpr int G = 8;
    const int kc1 = min(kc0 + p.kce, p.K);
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const int lo = part == 0 ? kc0 : max(kc0, p.k0);
      const int hi = part == 0 ? min(kc1, p.k0) : kc1;
      if (lo >= hi) continue;
      const float* base = part == 0 ? p.a0 + lo : p.a1 + (lo - p.k0);
      const int64_t ld = part == 0 ? p.lda0 : p.lda1;
      const int vpr = (hi - lo) / 4;
      const int nv = BM * vpr;
      for (int v0 = 0; v0 < nv; v0 += G * kBlock) {
        f4v st[G];
#pragma unroll
        for (int i = 0; i < G; ++i) {
          const int v = v0 + threadIdx.x + i * kBlock;
          const int r = v / vpr;
          const int64_t row = min(m0 + min(r, BM - 1), p.M - 1);
          st[i] = *reinterpret_cast<const f4v*>(base + row * ld + (v - r * vpr) * 4);
        }
#pragma unroll
        for (int i = 0; i < G; ++i) {
          const int v = v0 + threadIdx.x + i * kBlock;
          const int r = v / vpr;
          if (v < nv) {
            const float f[4] = {st[i][0], st[i][1], st[i][2], st[i][3]};
            uint2 h, md, l;
            sldm::split3_bf16x4(f, h, md, l);
            const int off = r * pa + (lo - kc0) + (v - r * vpr) * 4;
            *reinterpret_cast<uint2*>(img_hi + off) = h;
            *reinterpret_cast<uint2*>(img_mid + off) = md;
            *reinterpret_cast<uint2*>(img_lo + off) = l;
          }
        }
      }
    }
    __syncthreads();
    const int kend = kc1 - kc0;                         // a multiple of 32
    // weight fragments: 8 consecutive k of column bcol[t] per lane, fetched
    // one k-step ahead (two register sets), split on use
    f4v bx[TPW][2], by[TPW][2];
    auto loadb = [&](f4v (&bb)[TPW][2], int k) {
      const int ks = min(k, kend - 32);
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const float* src = p.b + (int64_t)bcol[t] * p.ldb + kc0 + ks + 8 * q;
        bb[t][0] = *reinterpret_cast<const f4v*>(src);
        bb[t][1] = *reinterpret_cast<const f4v*>(src + 4);
      }
    };
    auto mma = [&](f4v (&bb)[TPW][2], int k) {
      if (k >= kend) return;
      s8v ahi[MT], amid[MT], alo[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int off = (16 * m + r16) * pa + k + 8 * q;
        ahi[m] = *reinterpret_cast<const s8v*>(img_hi + off);
        amid[m] = *reinterpret_cast<const s8v*>(img_mid + off);
        alo[m] = *reinterpret_cast<const s8v*>(img_lo + off);
      }
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        if (!tval[t]) continue;
        const float w[8] = {bb[t][0][0], bb[t][0][1], bb[t][0][2], bb[t][0][3],
                            bb[t][1][0], bb[t][1][1], bb[t][1][2], bb[t][1][3]};
        s8v whi, wmid, wlo;
        sldm::split3_bf16x8(w, whi, wmid, wlo);
#pragma unroll
        for (int m = 0; m < MT; ++m)
          SLDM_MFMA_X6(acc[m][t], ahi[m], amid[m], alo[m], whi, wmid, wlo);
      }
    };
    loadb(bx, 0);
    for (int k0 = 0; k0 < kend; k0 += 64) {
      loadb(by, k0 + 32);
      mma(bx, k0);
      if (k0 + 32 >= kend) break;
      loadb(bx, k0 + 64);
      mma(by, k0 + 32);
    }
  }
  __syncthreads();  // LDS now holds the C tile

  const int ldc = 16 * p.ct + 4;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    if (!tval[t]) continue;
    const int c = 16 * (wave + 4 * t) + r16;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) smem[(16 * m + 4 * q + r) * ldc + c] = acc[m][t][r];
  }
  __syncthreads();

  nt_row_epilogue<float, MODE>(p, smem, ldc, m0, n0, BM, wave, lane);
}

// fp32 weight-stationary NT (exact-fp32 LN forward and dX with one column
// block, Nc <= 256, K = KC in {128, 256}; C2's shapes).  The tile kernel above
// re-reads its weight fragments from L2 every k-step and stages each A tile
// with a full load -> barrier -> compute sequence, so its MFMAs idle while
// loads are in flight (PMC: ~30 % MFMA-busy).  Here every wave loads its
// weight fragments once (<= 128 VGPRs) and the block walks 32-row tiles
// persistently: the next tile's A loads are issued right after the current
// tile lands in LDS and stay in flight under the MFMAs, which touch no
// vector memory.  Same k and sub-step order per accumulator as the tile
// kernel: bit-identical outputs.
template <int TPW, int KC, int MODE>
__global__ __launch_bounds__(kBlock, 2) void gemm_nt_ws32_kernel(NtArgs<float> p,
                                                                  int64_t ntiles) {
  using O = NtOps<float>;
  constexpr int MT = 2, BM = 32;
  constexpr int KSTEPS = KC / O::KS;
  constexpr int VPR = KC / 4;               // 16-B vectors per A row
  constexpr int NV = BM * VPR / kBlock;     // per thread per tile
  static_assert(BM * VPR % kBlock == 0 && KSTEPS * TPW <= 32, "ws32 shape");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int PA = KC + 4;                // A row pitch (floats): 16 B mod 256 B
  float* lds_a = smem;
  float* lds_c = smem + BM * PA;
  const int ldc = 16 * p.ct + 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, r16 = lane & 15;

  int64_t tile = blockIdx.x;
  if (tile >= ntiles) return;

  bool tval[TPW];
  f4v bw[KSTEPS][TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tid = wave + 4 * t;
    tval[t] = tid < p.ct;
    const int c = 16 * tid + r16;
    const int bc = c < p.Nc ? c : p.Nc - 1;
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) bw[ks][t] = nt_load_b<float, true>(p, bc, ks * O::KS + 4 * q);
  }

  f4v st[NV];
  auto load_tile = [&](int64_t tl) {
    const int64_t m0 = tl * BM;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = threadIdx.x + i * kBlock;
      const int r = v / VPR, kv = (v - r * VPR) * 4;
      const int64_t row = min(m0 + r, p.M - 1);
      const float* src = kv < p.k0 ? p.a0 + row * p.lda0 + kv : p.a1 + row * p.lda1 + (kv - p.k0);
      st[i] = *reinterpret_cast<const f4v*>(src);
    }
  };
  load_tile(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    // lds_a is free: every wave passed the barrier after the previous tile's MFMAs
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = threadIdx.x + i * kBlock;
      const int r = v / VPR, kv = (v - r * VPR) * 4;
      *reinterpret_cast<f4v*>(lds_a + r * PA + kv) = st[i];
    }
    __syncthreads();
    if (tile + gridDim.x < ntiles) load_tile(tile + gridDim.x);

    f4v acc[MT][TPW];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[m][t] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      f4v a[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m)
        a[m] = *reinterpret_cast<const f4v*>(lds_a + (16 * m + r16) * PA + ks * O::KS + 4 * q);
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        if (!tval[t]) continue;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m][c], bw[ks][t][c], acc[m][t], 0, 0, 0);
      }
    }
    // lds_c is free: every wave passed this tile's first barrier after its
    // previous epilogue
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (!tval[t]) continue;
      const int c = 16 * (wave + 4 * t) + r16;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) lds_c[(16 * m + 4 * q + r) * ldc + c] = acc[m][t][r];
    }
    __syncthreads();
    nt_row_epilogue<float, MODE>(p, lds_c, ldc, tile * BM, 0, BM, wave, lane);
  }
}

template <int TP, int KCV, int MODE>
int launch_ws32_t(const NtArgs<float>& p, int64_t ntiles, int64_t grid, size_t lds,
                  hipStream_t stream) {
  auto kern = gemm_nt_ws32_kernel<TP, KCV, MODE>;
  if (lds > 65536)
    SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, kBlock, lds, stream>>>(p, ntiles);
  SLDM_LAUNCH_CHECK("gemm_nt_ws32_kernel");
  return SLDM_OK;
}

// Returns -1 when the shape is not one the fp32 weight-stationary kernel takes
// (the tile kernel runs it), else the launch status.  SLDM_NT_WS32=0 disables.
template <int MODE>
int launch_nt_ws32(const NtArgs<float>& p, int tpw, hipStream_t stream) {
  const char* e = getenv("SLDM_NT_WS32");
  const bool enabled = !(e && e[0] == '0');
  auto mis = [](const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) != 0; };
  if (!enabled || p.M <= 0 || p.grid_y != 1 || !(p.K == 128 || p.K == 256) || p.k0 % 4 ||
      p.lda0 % 4 || p.lda1 % 4 || p.ldb % 4 || mis(p.a0) || (p.K > p.k0 && mis(p.a1)) || mis(p.b))
    return -1;
  const int64_t ntiles = (p.M + 31) / 32;
  const int64_t grid = ntiles < 512 ? ntiles : 512;   // 2 blocks x 256 CUs, persistent
  const size_t lds = sizeof(float) * (32 * (size_t)(p.K + 4) + 32 * (size_t)(16 * p.ct + 4));
  if (p.K == 256 && tpw == 1) return launch_ws32_t<1, 256, MODE>(p, ntiles, grid, lds, stream);
  if (p.K == 256 && tpw == 2) return launch_ws32_t<2, 256, MODE>(p, ntiles, grid, lds, stream);
  if (p.K == 128 && tpw == 1) return launch_ws32_t<1, 128, MODE>(p, ntiles, grid, lds, stream);
  if (p.K == 128 && tpw == 2) return launch_ws32_t<2, 128, MODE>(p, ntiles, grid, lds, stream);
  if (p.K == 128 && tpw == 3) return launch_ws32_t<3, 128, MODE>(p, ntiles, grid, lds, stream);
  if (p.K == 128 && tpw == 4) return launch_ws32_t<4, 128, MODE>(p, ntiles, grid, lds, stream);
  return -1;
}

template <typename T, int TPW, bool VEC, int MODE>
int launch_nt_t(const NtArgs<T>& p, hipStream_t stream) {
  constexpr int MT = NtTile<T>::MT;
  constexpr int BM = 16 * MT;
  int64_t nrb = (p.M + BM - 1) / BM;
  if (p.grid_y > 1) nrb = (nrb + 7) / 8 * 8;  // XCD mapping pads to a multiple of 8
  const int64_t grid = nrb * p.grid_y;
  SLDM_REQUIRE(grid < ((int64_t)1 << 31), "gemm_nt: grid too large");
  const size_t lds_c = sizeof(float) * (size_t)BM * (size_t)(16 * p.ct + 4);
  const size_t lds_a = sizeof(T) * (size_t)BM * (size_t)(p.kce + 16 / sizeof(T));
  const size_t lds = lds_c > lds_a ? lds_c : lds_a;
  auto kern = gemm_nt_kernel<T, MT, TPW, VEC, MODE>;
  if (lds > 65536)
    SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, kBlock, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("gemm_nt_kernel");
  return SLDM_OK;
}

template <int TPW, int MODE>
int launch_nt_x6_t(const NtArgs<float>& p, hipStream_t stream) {
  constexpr int MT = 4, BM = 16 * MT;
  int64_t nrb = (p.M + BM - 1) / BM;
  if (p.grid_y > 1) nrb = (nrb + 7) / 8 * 8;
  const int64_t grid = nrb * p.grid_y;
  SLDM_REQUIRE(grid < ((int64_t)1 << 31), "gemm_nt: grid too large");
  const size_t lds_c = sizeof(float) * (size_t)BM * (size_t)(16 * p.ct + 4);
  const size_t lds_a = 3 * sizeof(uint16_t) * (size_t)BM * (size_t)(p.kce + 8);
  const size_t lds = lds_c > lds_a ? lds_c : lds_a;
  auto kern = gemm_nt_x6_kernel<MT, TPW, MODE>;
  if (lds > 65536)
    SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, kBlock, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("gemm_nt_x6_kernel");
  return SLDM_OK;
}

template <typename T, int MODE>
int launch_nt(NtArgs<T>& p, hipStream_t stream) {
  constexpr int EPL = NtOps<T>::EPL;
  constexpr int KS = NtOps<T>::KS;
  const int total_ct = (p.Nc + 15) / 16;
  if (MODE == EPI_LN) {
    SLDM_REQUIRE(total_ct <= 16, "sldm_sage_dense_fwd: F_out=%d > 256 unsupported", p.Nc);
    p.ct = total_ct;
    p.grid_y = 1;
  } else {
    p.ct = total_ct < 16 ? total_ct : 16;
    p.grid_y = (total_ct + p.ct - 1) / p.ct;
  }
  // K chunk staged per pass: up to 1 KiB of a row, a multiple of the k-step.
  const int kmax = 1024 / (int)sizeof(T);
  const int kround = (p.K + KS - 1) / KS * KS;
  p.kce = kround < kmax ? kround : kmax;
  auto al = [](const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; };
  const int k1 = p.K - p.k0;
  const bool vec = (p.k0 % EPL == 0) && (k1 % EPL == 0) && (p.lda0 % EPL == 0) &&
                   (k1 == 0 || p.lda1 % EPL == 0) && (p.ldb % EPL == 0) && al(p.a0) &&
                   (k1 == 0 || al(p.a1)) && al(p.b) && (p.K % KS == 0);
  const int tpw = (p.ct + 3) / 4;
  if constexpr (sizeof(T) == 4) {
    // split-bf16 products for the vector shapes (K a multiple of 32)
    if (vec && p.K % 32 == 0 && p.kce % 32 == 0 && sldm::fp32_gemm_split()) {
      // 128-deep K chunks: the three staged images stay below the C tile's
      // LDS footprint (two blocks per CU)
      NtArgs<float> q = p;
      q.kce = p.kce < 128 ? p.kce : 128;
      switch (tpw) {
        case 1: return launch_nt_x6_t<1, MODE>(q, stream);
        case 2: return launch_nt_x6_t<2, MODE>(q, stream);
        case 3: return launch_nt_x6_t<3, MODE>(q, stream);
        case 4: return launch_nt_x6_t<4, MODE>(q, stream);
      }
    }
    // exact fp32 MFMA: the weight-stationary kernel where its shape fits
    const int rc = launch_nt_ws32<MODE>(p, tpw, stream);
    if (rc >= 0) return rc;
  }
#define SLDM_NT_CASE(TP)                                                        \
  case TP:                                                                      \
    return vec ? launch_nt_t<T, TP, true, MODE>(p, stream)                      \
               : launch_nt_t<T, TP, false, MODE>(p, stream);
  switch (tpw) {
    SLDM_NT_CASE(1)
    SLDM_NT_CASE(2)
    SLDM_NT_CASE(3)
    SLDM_NT_CASE(4)
  }
#undef SLDM_NT_CASE
  sldm::set_error("gemm_nt: bad tile count %d", tpw);
  return SLDM_ERR_ARG;
}

// ------------------------------------------------------------------- TN --
#ifndef SLDM_TN_BK
#define SLDM_TN_BK 32
#endif
template <typename T>
struct TnArgs {
  const T* a; int64_t lda; int mo;             // A [rows][mo]
  const T* b0; int64_t ldb0; int n0;           // B columns [0, n0)
  const T* b1; int64_t ldb1; int nn;           // B columns [n0, nn)
  int64_t rows;                                // the summed (node) dimension
  int64_t chunk;                               // rows per split (multiple of 32)
  int splits, tiles_m, tiles_n;
  float* slab;                                 // [splits][mo][nn]
};

constexpr int TN_BK = SLDM_TN_BK;   // node rows per k-step (32 | 64)
constexpr int TN_TILE = 128; // block tile (m and n)

template <typename T> struct TnLds {
  // row pitch (elements) of a [TN_BK][TN_TILE] staging tile; 32-byte pad
  static constexpr int pitch = TN_TILE + 32 / (int)sizeof(T);
};

// Stage rows [k0, k0+32) x cols [c0, c0+128) of a row-major operand into
// registers (16 B per lane-load, coalesced along rows).
template <typename T, bool VEC>
struct TnStage {
  static constexpr int EPV = 16 / sizeof(T);                         // elems per vector
  static constexpr int NV = TN_BK * TN_TILE / EPV / kBlock;          // vectors per thread
  uint4 v[NV];

  template <class Elem>
  __device__ void load(Elem elem, int64_t k0, int c0, int64_t kend, int cend) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = threadIdx.x + i * kBlock;
      const int r = idx / (TN_TILE / EPV);
      const int cv = (idx % (TN_TILE / EPV)) * EPV;
      const int64_t k = k0 + r;
      const int c = c0 + cv;
      if constexpr (VEC) {
        const int64_t kc = k < kend ? k : kend - 1;
        const int cc = c < cend ? c : cend - EPV;
        uint4 x = *reinterpret_cast<const uint4*>(elem(kc, cc));
        if (k >= kend || c >= cend) x = make_uint4(0, 0, 0, 0);
        v[i] = x;
      } else {
        T tmp[EPV];
#pragma unroll
        for (int j = 0; j < EPV; ++j) {
          const int cj = c + j;
          const int64_t kc = k < kend ? k : kend - 1;
          const int cc = cj < cend ? cj : cend - 1;
          T x = *elem(kc, cc);
          tmp[j] = (k < kend && cj < cend) ? x : (T)0;
        }
        v[i] = *reinterpret_cast<const uint4*>(tmp);
      }
    }
  }
  __device__ void store(T* lds) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = threadIdx.x + i * kBlock;
      const int r = idx / (TN_TILE / EPV);
      const int cv = (idx % (TN_TILE / EPV)) * EPV;
      *reinterpret_cast<uint4*>(lds + r * TnLds<T>::pitch + cv) = v[i];
    }
  }
};

template <typename T, bool VEC>
__global__ __launch_bounds__(kBlock) void gemm_tn_kernel(TnArgs<T> p) {
  __shared__ __attribute__((aligned(16))) T lds[2 * TN_BK * TnLds<T>::pitch];
  T* lds_a = lds;
  T* lds_b = lds + TN_BK * TnLds<T>::pitch;
  constexpr int PITCH = TnLds<T>::pitch;

  // blockIdx -> (split, tile): the tiles of one split share blockIdx % 8
  // (one XCD under round-robin dispatch; speed only).
  const int b = blockIdx.x;
  const int tiles = p.tiles_m * p.tiles_n;
  int split, tile;
  if (p.splits % 8 == 0) {
    const int xcd = b % 8, j = b / 8;
    tile = j % tiles;
    split = (j / tiles) * 8 + xcd;
  } else {
    tile = b % tiles;
    split = b / tiles;
  }
  const int tm = tile / p.tiles_n, tn = tile % p.tiles_n;
  const int mbase = tm * TN_TILE, nbase = tn * TN_TILE;
  const int64_t kbeg = (int64_t)split * p.chunk;
  const int64_t kend = min(kbeg + p.chunk, p.rows);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;   // 2 x 2 waves, 64 x 64 each

  f4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  auto elem_a = [&](int64_t k, int c) { return p.a + k * p.lda + c; };
  auto elem_b = [&](int64_t k, int c) {
    return c < p.n0 ? p.b0 + k * p.ldb0 + c : p.b1 + k * p.ldb1 + (c - p.n0);
  };
  TnStage<T, VEC> sa, sb;
  if (kbeg < kend) {
    sa.load(elem_a, kbeg, mbase, kend, p.mo);
    sb.load(elem_b, kbeg, nbase, kend, p.nn);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += TN_BK) {
    __syncthreads();
    sa.store(lds_a);
    sb.store(lds_b);
    __syncthreads();
    if (k0 + TN_BK < kend) {
      sa.load(elem_a, k0 + TN_BK, mbase, kend, p.mo);
      sb.load(elem_b, k0 + TN_BK, nbase, kend, p.nn);
    }
    if constexpr (sizeof(T) == 2) {
#pragma unroll
     for (int kb = 0; kb < TN_BK; kb += 32) {
      // Lane 4i+j of a 16-lane group addresses row (8q + i), columns 4j..4j+3
      // of a 4x16 block; it receives column r16 of rows 8q..8q+3 (T10).
      const int rr = kb + 8 * q + (r16 >> 2);
      const int cc = 4 * (r16 & 3);
      s8v af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const T* pa = lds_a + rr * PITCH + wm * 64 + 16 * i + cc;
        s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4v*)(pa));
        s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4v*)(pa + 4 * PITCH));
        af[i] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const T* pb = lds_b + rr * PITCH + wn * 64 + 16 * i + cc;
        lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(pb));
        hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4v*)(pb + 4 * PITCH));
        bf[i] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
     }
    } else {
#pragma unroll
      for (int kk = 0; kk < TN_BK; kk += 4) {
        float af[4], bf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          af[i] = reinterpret_cast<const float*>(lds_a)[(kk + q) * PITCH + wm * 64 + 16 * i + r16];
          bf[i] = reinterpret_cast<const float*>(lds_b)[(kk + q) * PITCH + wn * 64 + 16 * i + r16];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  // Partial tile -> slab[split] (C map: col = r16, row = 4q + r).
  float* out = p.slab + (int64_t)split * p.mo * p.nn;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = nbase + wn * 64 + 16 * j + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mbase + wm * 64 + 16 * i + 4 * q + r;
        if (row < p.mo && col < p.nn) out[(int64_t)row * p.nn + col] = acc[i][j][r];
      }
    }
}

// The fp32 TN kernel with split-bf16 products (see gemm_nt_x6_kernel): both
// staged operand tiles become hi / mid / lo bf16 images in LDS as they are
// stored, and the MFMA phase is the bf16 kernel's transposed reads with the
// six-term product per accumulator and 32-row k-step instead of eight exact
// 16x16x4 fp32 MFMAs.  16-B aligned operands.
__global__ __launch_bounds__(kBlock) void gemm_tn_x6_kernel(TnArgs<float> p) {
  constexpr int PITCH = TnLds<uint16_t>::pitch;
  __shared__ __attribute__((aligned(16))) uint16_t lds[6 * TN_BK * PITCH];
  uint16_t* a_hi = lds;
  uint16_t* a_mid = lds + TN_BK * PITCH;
  uint16_t* a_lo = lds + 2 * TN_BK * PITCH;
  uint16_t* b_hi = lds + 3 * TN_BK * PITCH;
  uint16_t* b_mid = lds + 4 * TN_BK * PITCH;
  uint16_t* b_lo = lds + 5 * TN_BK * PITCH;

  const int b = blockIdx.x;
  const int tiles = p.tiles_m * p.tiles_n;
  int split, tile;
  if (p.splits % 8 == 0) {
    const int xcd = b % 8, j = b / 8;
    tile = j % tiles;
    split = (j / tiles) * 8 + xcd;
  } else {
    tile = b % tiles;
    split = b / tiles;
  }
  const int tm = tile / p.tiles_n, tn = tile % p.tiles_n;
  const int mbase = tm * TN_TILE, nbase = tn * TN_TILE;
  const int64_t kbeg = (int64_t)split * p.chunk;
  const int64_t kend = min(kbeg + p.chunk, p.rows);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, r16 = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;

  f4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  auto elem_a = [&](int64_t k, int c) { return p.a + k * p.lda + c; };
  auto elem_b = [&](int64_t k, int c) {
    return c < p.n0 ? p.b0 + k * p.ldb0 + c : p.b1 + k * p.ldb1 + (c - p.n0);
  };
  using Stage = TnStage<float, true>;
  auto store_split = [&](const Stage& st, uint16_t* hi, uint16_t* mid, uint16_t* lo) {
#pragma unroll
    for (int i = 0; i < Stage::NV; ++i) {
      const int idx = threadIdx.x + i * kBlock;
      const int r = idx / (TN_TILE / 4);
      const int cv = (idx % (TN_TILE / 4)) * 4;
      const float f[4] = {__uint_as_float(st.v[i].x), __uint_as_float(st.v[i].y),
                          __uint_as_float(st.v[i].z), __uint_as_float(st.v[i].w)};
      uint2 h, md, l;
      sldm::split3_bf16x4(f, h, md, l);
      *reinterpret_cast<uint2*>(hi + r * PITCH + cv) = h;
      *reinterpret_cast<uint2*>(mid + r * PITCH + cv) = md;
      *reinterpret_cast<uint2*>(lo + r * PITCH + cv) = l;
    }
  };
  auto read_tr = [&](const uint16_t* img, int rr, int col) {
    const uint16_t* pa = img + rr * PITCH + col;
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s4v*)(pa));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s4v*)(pa + 4 * PITCH));
    return s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  Stage sa, sb;
  if (kbeg < kend) {
    sa.load(elem_a, kbeg, mbase, kend, p.mo);
    sb.load(elem_b, kbeg, nbase, kend, p.nn);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += TN_BK) {
    __syncthreads();
    store_split(sa, a_hi, a_mid, a_lo);
    store_split(sb, b_hi, b_mid, b_lo);
    __syncthreads();
    if (k0 + TN_BK < kend) {
      sa.load(elem_a, k0 + TN_BK, mbase, kend, p.mo);
      sb.load(elem_b, k0 + TN_BK, nbase, kend, p.nn);
    }
#pragma unroll
    for (int kb = 0; kb < TN_BK; kb += 32) {
      const int rr = kb + 8 * q + (r16 >> 2);
      const int cc = 4 * (r16 & 3);
      s8v ah[4], am[4], al[4], bh[4], bm[4], bl[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ah[i] = read_tr(a_hi, rr, wm * 64 + 16 * i + cc);
        am[i] = read_tr(a_mid, rr, wm * 64 + 16 * i + cc);
        al[i] = read_tr(a_lo, rr, wm * 64 + 16 * i + cc);
        bh[i] = read_tr(b_hi, rr, wn * 64 + 16 * i + cc);
        bm[i] = read_tr(b_mid, rr, wn * 64 + 16 * i + cc);
        bl[i] = read_tr(b_lo, rr, wn * 64 + 16 * i + cc);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          SLDM_MFMA_X6(acc[i][j], ah[i], am[i], al[i], bh[j], bm[j], bl[j]);
    }
  }

  float* out = p.slab + (int64_t)split * p.mo * p.nn;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = nbase + wn * 64 + 16 * j + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mbase + wm * 64 + 16 * i + 4 * q + r;
        if (row < p.mo && col < p.nn) out[(int64_t)row * p.nn + col] = acc[i][j][r];
      }
    }
}

// out1 != nullptr: element (row, col) of the [mo, nn] result goes to out
// [mo, n0] for col < n0 and to out1 [mo, nn - n0] otherwise (dW_l, dW_r).
__global__ __launch_bounds__(kBlock) void slab_reduce_kernel(const float* __restrict__ slab,
                                                             int splits, int64_t n,
                                                             float* __restrict__ out,
                                                             float* __restrict__ out1, int64_t n0,
                                                             int64_t nn) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  // Sum over the splits in split order (deterministic, fixed bits); the loads
  // go out 32 at a time ahead of the in-order adds -- one load round trip per
  // 32 splits instead of one per split (C2 fp32 dW, 256 splits: 60 -> 6.3 us).
  constexpr int U = 32;
  float s = 0.f;
  int k = 0;
  for (; k + U <= splits; k += U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = slab[(int64_t)(k + u) * n + i];
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  for (; k < splits; ++k) s += slab[(int64_t)k * n + i];
  if (out1) {
    const int64_t row = i / nn, col = i - row * nn;
    if (col < n0) out[row * n0 + col] = s;
    else out1[row * (nn - n0) + (col - n0)] = s;
  } else {
    out[i] = s;
  }
}

struct TnPlan {
  int splits, tiles_m, tiles_n;
  int64_t chunk;
};

// ``x6``: the plan of the fp32 split-bf16 kernel (two resident blocks per CU).
TnPlan tn_plan(int64_t rows, int64_t mo, int64_t nn, bool x6 = false) {
  TnPlan pl;
  pl.tiles_m = (int)((mo + TN_TILE - 1) / TN_TILE);
  pl.tiles_n = (int)((nn + TN_TILE - 1) / TN_TILE);
  const int tiles = pl.tiles_m * pl.tiles_n;
  // ~3 resident blocks per CU (the kernel runs 3 waves per SIMD) on long node
  // dimensions; the SLDM_TN_BLOCKS environment variable overrides (A/B runs)
  static const int64_t target = [] {
    const char* e = getenv("SLDM_TN_BLOCKS");
    const long v = e ? atol(e) : 0;
    return (int64_t)(v > 0 ? v : 0);
  }();
  // 768 measured best at C4 (10M rows: 4.63 -> 3.84 ms vs 512); short node
  // dimensions keep 512 (C2: the extra slabs cost more than they hide)
  // the split-bf16 fp32 kernel holds six LDS images (two blocks per CU): 1024
  // blocks = two full rounds (C4 dW 16.9 -> 15.5 ms against 768)
  int64_t splits = (target ? target : (rows >= 2000000 ? (x6 ? 1024 : 768) : 512)) / tiles;
  // >= 8 k-steps per split on long node dimensions; short ones (the vehicle
  // batches' ~8k rows: 31 splits = 48 blocks of 11 k-steps, 40 us of mostly
  // idle CUs) take more, shorter splits; SLDM_TN_MINK overrides (A/B runs)
  static const int64_t mink_env = [] {
    const char* e = getenv("SLDM_TN_MINK");
    const long v = e ? atol(e) : 0;
    return (int64_t)(v > 0 ? v : 0);
  }();
  const int64_t mink = mink_env ? mink_env : (rows >= 65536 ? 8 : 3);
  const int64_t max_splits = (rows + mink * TN_BK - 1) / (mink * TN_BK);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  if (splits >= 8) splits = (splits / 8) * 8;
  int64_t chunk = (rows + splits - 1) / splits;
  chunk = (chunk + TN_BK - 1) / TN_BK * TN_BK;
  if (chunk < TN_BK) chunk = TN_BK;
  pl.splits = (int)splits;
  pl.chunk = chunk;
  return pl;
}

}  // namespace

// ------------------------------------------------------------------ C ABI --
extern "C" int sldm_sage_dense_fwd(int dtype, const void* a0, int64_t lda0, int64_t k0,
                                   const void* a1, int64_t lda1, int64_t k1, const void* w,
                                   int64_t num_rows, int64_t nc, const float* bias,
                                   const float* gamma, const float* beta, float eps,
                                   float negative_slope, float drop_p, uint64_t seed,
                                   int64_t row_off, void* out,
                                   void* xhat, float* rstd, void* stream_) {
  SLDM_REQUIRE(dtype == SLDM_F32 || dtype == SLDM_BF16, "sldm_sage_dense_fwd: dtype %d", dtype);
  SLDM_REQUIRE(num_rows >= 0 && k0 >= 0 && k1 >= 0 && k0 + k1 > 0 && nc > 0 && nc <= 256,
               "sldm_sage_dense_fwd: bad sizes (k0=%lld k1=%lld nc=%lld)", (long long)k0,
               (long long)k1, (long long)nc);
  SLDM_REQUIRE(drop_p >= 0.f && drop_p <= 1.f, "sldm_sage_dense_fwd: drop_p=%g", (double)drop_p);
  if (num_rows == 0) return SLDM_OK;
  SLDM_REQUIRE(a0 && w && out && gamma && beta && (k1 == 0 || a1),
               "sldm_sage_dense_fwd: NULL argument");
  hipStream_t stream = sldm::as_stream(stream_);
  if (dtype == SLDM_BF16 && sldm::stream_gemm_enabled() &&
      sldm::stream_dense_fwd_ok(k0, k0 + k1, nc, a0, lda0, k1 ? a1 : a0, k1 ? lda1 : lda0, w,
                                out, xhat, negative_slope))
    return sldm::stream_dense_fwd(a0, lda0, k0, a1, lda1, k1, w, num_rows, bias, gamma, beta,
                                  eps, negative_slope, drop_p, seed, row_off, out, xhat, rstd,
                                  stream);
  if (dtype == SLDM_BF16 && sldm::big_gemm_enabled() && (nc == 128 || nc == 256) &&
      sldm::big_gemm_ok(k0, k0 + k1, nc, a0, lda0, k1 ? a1 : a0, k1 ? lda1 : lda0, w, k0 + k1,
                        nc))
    return sldm::big_dense_fwd(a0, lda0, k0, a1, lda1, k1, w, num_rows, nc, bias, gamma, beta,
                               eps, negative_slope, drop_p, seed, row_off, out, xhat, rstd,
                               stream);
  if (dtype == SLDM_F32 && sldm::fp32_gemm_split() && sldm::stream_f32_enabled() &&
      sldm::stream_f32_dense_fwd_ok(k0, k0 + k1, nc, a0, lda0, k1 ? a1 : a0, k1 ? lda1 : lda0, w,
                                    out, xhat))
    return sldm::stream_f32_dense_fwd(a0, lda0, k0, a1, lda1, k1, w, num_rows, bias, gamma, beta,
                                      eps, negative_slope, drop_p, seed, row_off, out, xhat, rstd,
                                      stream);
  auto fill = [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    NtArgs<T> p{};
    p.a0 = (const T*)a0; p.lda0 = lda0; p.k0 = (int)k0;
    p.a1 = k1 ? (const T*)a1 : (const T*)a0; p.lda1 = k1 ? lda1 : lda0;
    p.K = (int)(k0 + k1);
    p.b = (const T*)w; p.ldb = k0 + k1;
    p.M = num_rows; p.Nc = (int)nc;
    p.out = (T*)out; p.ldo = nc; p.xhat = (T*)xhat; p.rstd = rstd;
    p.bias = bias; p.gamma = gamma; p.beta = beta; p.eps = eps; p.slope = negative_slope;
    p.drop_p = drop_p;
    p.drop_scale = drop_p >= 1.f ? 0.f : (drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f);
    p.seed = seed;
    p.row_off = row_off;
    return launch_nt<T, EPI_LN>(p, stream);
  };
  return dtype == SLDM_F32 ? fill((float*)nullptr) : fill((uint16_t*)nullptr);
}

extern "C" int sldm_gemm_nt_rowscale(int dtype, const void* a, int64_t lda, int64_t k,
                                     const void* b, int64_t ldb, int64_t num_rows, int64_t nc,
                                     const int32_t* rowptr, int64_t scale_cols, void* out,
                                     int64_t ldo, void* out2, int64_t ldo2, void* stream_) {
  SLDM_REQUIRE(dtype == SLDM_F32 || dtype == SLDM_BF16, "sldm_gemm_nt_rowscale: dtype %d", dtype);
  SLDM_REQUIRE(num_rows >= 0 && k > 0 && nc > 0 && lda >= k && ldb >= k,
               "sldm_gemm_nt_rowscale: bad sizes");
  if (out2) {
    SLDM_REQUIRE(scale_cols > 0 && scale_cols < nc && scale_cols % 4 == 0 &&
                     ldo >= scale_cols && ldo2 >= nc - scale_cols,
                 "sldm_gemm_nt_rowscale: split output needs 0 < scale_cols < nc, "
                 "scale_cols %% 4 == 0 and ld >= the half widths");
  } else {
    SLDM_REQUIRE(ldo >= nc, "sldm_gemm_nt_rowscale: ldo < nc");
  }
  if (num_rows == 0) return SLDM_OK;
  SLDM_REQUIRE(a && b && out, "sldm_gemm_nt_rowscale: NULL argument");
  hipStream_t stream = sldm::as_stream(stream_);
  if (dtype == SLDM_BF16 && sldm::ws_gemm_enabled() &&
      sldm::ws_rowscale_ok(k, nc, num_rows, a, lda, b, ldb, out, ldo, out2, ldo2,
                           rowptr || out2 ? scale_cols : 0))
    return sldm::ws_gemm_rowscale(a, lda, k, b, ldb, num_rows, nc, rowptr, scale_cols, out, ldo,
                                  out2, ldo2, stream);
  if (dtype == SLDM_BF16 && sldm::stream_gemm_enabled() &&
      sldm::stream_rowscale_ok(k, nc, a, lda, b, ldb, out, ldo, scale_cols) &&
      (!out2 || (ldo2 == ldo && scale_cols % 256 == 0 &&
                 sldm::stream_rowscale_ok(k, nc, a, lda, b, ldb, out2, ldo2, scale_cols))))
    return sldm::stream_gemm_rowscale(a, lda, k, b, ldb, num_rows, nc, rowptr, scale_cols, out,
                                      ldo, out2, ldo2, stream);
  if (dtype == SLDM_BF16 && sldm::big_gemm_enabled() && nc % 128 == 0) {
    const int64_t bn = nc % 256 == 0 ? 256 : 128;
    if (sldm::big_gemm_ok(k, k, bn, a, lda, a, lda, b, ldb, out2 ? 4 : ldo) &&
        (!out2 || (ldo % 4 == 0 && ldo2 % 4 == 0)))
      return sldm::big_gemm_rowscale(a, lda, k, b, ldb, num_rows, nc, bn, rowptr, scale_cols,
                                     out, ldo, out2, ldo2, stream);
  }
  if (dtype == SLDM_F32 && sldm::fp32_gemm_split() && sldm::stream_f32_enabled() &&
      sldm::stream_f32_rowscale_ok(k, nc, a, lda, b, ldb, out, ldo, out2, ldo2,
                                   rowptr || out2 ? scale_cols : 0))
    return sldm::stream_f32_gemm_rowscale(a, lda, k, b, ldb, num_rows, nc, rowptr, scale_cols,
                                          out, ldo, out2, ldo2, stream);
  auto fill = [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    NtArgs<T> p{};
    p.a0 = (const T*)a; p.lda0 = lda; p.k0 = (int)k;
    p.a1 = (const T*)a; p.lda1 = lda;
    p.K = (int)k;
    p.b = (const T*)b; p.ldb = ldb;
    p.M = num_rows; p.Nc = (int)nc;
    p.out = (T*)out; p.ldo = ldo;
    p.out2 = (T*)out2; p.ldo2 = ldo2;
    p.rowptr = rowptr; p.scale_cols = (int)scale_cols;
    return launch_nt<T, EPI_ROWSCALE>(p, stream);
  };
  return dtype == SLDM_F32 ? fill((float*)nullptr) : fill((uint16_t*)nullptr);
}

extern "C" int sldm_gemm_nt_rowscale_blocked_ok(int dtype, int64_t k, int64_t nc,
                                                int64_t scale_cols, int64_t blk_cols) {
  return dtype == SLDM_BF16 && sldm::ws_gemm_enabled() && k == 256 && nc == 512 &&
         scale_cols == 256 && (blk_cols == 32 || blk_cols == 64 || blk_cols == 128);
}

extern "C" int sldm_gemm_nt_rowscale_blocked(int dtype, const void* a, int64_t lda, int64_t k,
                                             const void* b, int64_t ldb, int64_t num_rows,
                                             int64_t nc, const int32_t* rowptr,
                                             int64_t scale_cols, void* out_blocked,
                                             int64_t blk_cols, void* out2, int64_t ldo2,
                                             void* stream_) {
  SLDM_REQUIRE(sldm_gemm_nt_rowscale_blocked_ok(dtype, k, nc, scale_cols, blk_cols),
               "sldm_gemm_nt_rowscale_blocked: unsupported shape (dtype %d k %lld nc %lld "
               "scale_cols %lld blk_cols %lld); ask sldm_gemm_nt_rowscale_blocked_ok first",
               dtype, (long long)k, (long long)nc, (long long)scale_cols, (long long)blk_cols);
  SLDM_REQUIRE(num_rows >= 0 && lda >= k && ldb >= k && ldo2 >= nc - scale_cols,
               "sldm_gemm_nt_rowscale_blocked: bad sizes");
  if (num_rows == 0) return SLDM_OK;
  SLDM_REQUIRE(a && b && out_blocked && out2, "sldm_gemm_nt_rowscale_blocked: NULL argument");
  SLDM_REQUIRE(sldm::ws_rowscale_ok(k, nc, num_rows, a, lda, b, ldb, out_blocked, blk_cols, out2,
                                    ldo2, scale_cols),
               "sldm_gemm_nt_rowscale_blocked: operands must be 16-byte aligned with row "
               "strides that are multiples of 8 elements");
  const int sh = blk_cols == 32 ? 5 : (blk_cols == 64 ? 6 : 7);
  return sldm::ws_gemm_rowscale(a, lda, k, b, ldb, num_rows, nc, rowptr, scale_cols, out_blocked,
                                blk_cols, out2, ldo2, sldm::as_stream(stream_), sh);
}

extern "C" size_t sldm_gemm_tn_workspace_bytes(int64_t num_rows, int64_t mo, int64_t nn) {
  if (num_rows <= 0 || mo <= 0 || nn <= 0) return 16;
  // no dtype here: room for the larger of the two plans
  const int splits = std::max(tn_plan(num_rows, mo, nn).splits, tn_plan(num_rows, mo, nn, true).splits);
  size_t need = sizeof(float) * (size_t)splits * (size_t)mo * (size_t)nn + 256;
  if (mo == 256 && (nn == 256 || nn == 512))   // gemm_tn_dma.hip's slab may be larger
    need = std::max(need, sldm::tn_dma_workspace_bytes(num_rows, nn));
  return need;
}

namespace {
int gemm_tn_impl(int dtype, const void* a, int64_t lda, int64_t mo, const void* b0, int64_t ldb0,
                 int64_t n0, const void* b1, int64_t ldb1, int64_t n1, int64_t num_rows,
                 float* out, float* out1, void* workspace, size_t ws_bytes, void* stream_) {
  SLDM_REQUIRE(dtype == SLDM_F32 || dtype == SLDM_BF16, "sldm_gemm_tn: dtype %d", dtype);
  SLDM_REQUIRE(mo > 0 && n0 >= 0 && n1 >= 0 && n0 + n1 > 0 && num_rows >= 0,
               "sldm_gemm_tn: bad sizes");
  SLDM_REQUIRE(a && b0 && out && (n1 == 0 || b1), "sldm_gemm_tn: NULL argument");
  hipStream_t stream = sldm::as_stream(stream_);
  const int64_t nn = n0 + n1;
  if (num_rows == 0) {
    if (!out1) return sldm::zero_words(out, (size_t)(mo * nn), stream);
    const int rc = sldm::zero_words(out, (size_t)(mo * n0), stream);
    return rc != SLDM_OK ? rc : sldm::zero_words(out1, (size_t)(mo * n1), stream);
  }
  const size_t need = sldm_gemm_tn_workspace_bytes(num_rows, mo, nn);
  SLDM_REQUIRE(workspace && ws_bytes >= need, "sldm_gemm_tn: workspace too small (%zu < %zu)",
               ws_bytes, need);
  float* slab = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(workspace) + 255) & ~(uintptr_t)255);
  if (dtype == SLDM_BF16 && sldm::tn_dma_enabled() &&
      sldm::tn_dma_ok(mo, n0, n1, num_rows, a, lda, b0, ldb0, b1, ldb1)) {
    int splits = 0;
    const int rc = sldm::tn_dma(a, lda, b0, ldb0, b1, ldb1, n1, num_rows, slab, &splits, stream);
    if (rc != SLDM_OK) return rc;
    const int64_t n = mo * nn;
    slab_reduce_kernel<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, stream>>>(
        slab, splits, n, out, out1, n0, nn);
    SLDM_LAUNCH_CHECK("slab_reduce_kernel");
    return SLDM_OK;
  }
  auto run = [&](auto* tag) -> int {
    using T = std::remove_pointer_t<decltype(tag)>;
    constexpr int EPV = 16 / sizeof(T);
    auto al = [](const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; };
    const bool vec = (mo % EPV == 0) && (n0 % EPV == 0) && (n1 % EPV == 0) && (lda % EPV == 0) &&
                     (ldb0 % EPV == 0) && (n1 == 0 || ldb1 % EPV == 0) && al(a) && al(b0) &&
                     (n1 == 0 || al(b1));
    const bool x6 = sizeof(T) == 4 && vec && sldm::fp32_gemm_split();
    const TnPlan pl = tn_plan(num_rows, mo, nn, x6);
    TnArgs<T> p{};
    p.a = (const T*)a; p.lda = lda; p.mo = (int)mo;
    p.b0 = (const T*)b0; p.ldb0 = ldb0; p.n0 = (int)n0;
    p.b1 = n1 ? (const T*)b1 : (const T*)b0; p.ldb1 = n1 ? ldb1 : ldb0; p.nn = (int)nn;
    p.rows = num_rows; p.chunk = pl.chunk; p.splits = pl.splits;
    p.tiles_m = pl.tiles_m; p.tiles_n = pl.tiles_n; p.slab = slab;
    const unsigned grid = (unsigned)(pl.splits * pl.tiles_m * pl.tiles_n);
    if constexpr (sizeof(T) == 4) {
      if (x6) gemm_tn_x6_kernel<<<grid, kBlock, 0, stream>>>(p);
    }
    if (x6) {
    } else if (vec)
      gemm_tn_kernel<T, true><<<grid, kBlock, 0, stream>>>(p);
    else
      gemm_tn_kernel<T, false><<<grid, kBlock, 0, stream>>>(p);
    SLDM_LAUNCH_CHECK("gemm_tn_kernel");
    const int64_t n = mo * nn;
    slab_reduce_kernel<<<(unsigned)((n + kBlock - 1) / kBlock), kBlock, 0, stream>>>(
        slab, pl.splits, n, out, out1, n0, nn);
    SLDM_LAUNCH_CHECK("slab_reduce_kernel");
    return SLDM_OK;
  };
  return dtype == SLDM_F32 ? run((float*)nullptr) : run((uint16_t*)nullptr);
}
}  // namespace

extern "C" int sldm_gemm_tn(int dtype, const void* a, int64_t lda, int64_t mo, const void* b0,
                            int64_t ldb0, int64_t n0, const void* b1, int64_t ldb1, int64_t n1,
                            int64_t num_rows, float* out, void* workspace, size_t ws_bytes,
                            void* stream_) {
  return gemm_tn_impl(dtype, a, lda, mo, b0, ldb0, n0, b1, ldb1, n1, num_rows, out, nullptr,
                      workspace, ws_bytes, stream_);
}

extern "C" int sldm_gemm_tn_split(int dtype, const void* a, int64_t lda, int64_t mo,
                                  const void* b0, int64_t ldb0, int64_t n0, const void* b1,
                                  int64_t ldb1, int64_t n1, int64_t num_rows, float* out0,
                                  float* out1, void* workspace, size_t ws_bytes, void* stream_) {
  SLDM_REQUIRE(n0 > 0 && n1 > 0 && out0 && out1, "sldm_gemm_tn_split: needs n0, n1 > 0 and both outputs");
  return gemm_tn_impl(dtype, a, lda, mo, b0, ldb0, n0, b1, ldb1, n1, num_rows, out0, out1,
                      workspace, ws_bytes, stream_);
}

namespace sldm {
// fp32 dense GEMMs run as six-term split-bf16 products (three-way operand
// split on the bf16 MFMA, fp32-level products, fp32 accumulation) wherever a
// kernel has that form; SLDM_FP32_GEMM=exact selects the exact fp32 MFMA
// (v_mfma_f32_16x16x4_f32, 1/16 of the bf16 rate) everywhere.  Read per call
// so tests can compare both forms in one process.
bool fp32_gemm_split() {
  const char* e = getenv("SLDM_FP32_GEMM");
  return !(e && e[0] == 'e');
}
}  // namespace sldm
