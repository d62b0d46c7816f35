// Big-tile bf16 MFMA kernels for the dense part of a SageBlock layer (the
// large-F_out shapes: F_out, or the column block, of 128 or 256).
//
// Same contractions and epilogues as gemm.hip (forward [agg|x]·W^T + bias +
// LayerNorm + act + dropout; backward dh·W with the 1/deg prescale), built the
// way an HBM-streaming GEMM wants to be on gfx950:
//
//  * block = 8 waves (512 threads) x a 256-row tile x all BN (128|256) columns,
//    so every weight element staged into LDS serves 256 rows and the LayerNorm
//    row statistics stay inside the block;
//  * operands stream global -> LDS by LDS-DMA (global_load_lds_dwordx4, no
//    VGPRs, no ds_write) through a 4-stage ring of 32-deep k-slices (64 B per
//    row per slice), prefetch distance 3, a counted `s_waitcnt vmcnt` and ONE
//    raw s_barrier per k-step (a __syncthreads would drain every DMA in flight);
//  * the LDS image is lane-linear per DMA instruction (16 rows x 64 B), the
//    16-B chunk of row R holding k-chunk c sits in slot c ^ ((R >> 2) & 2): the
//    swizzle goes on the SOURCE address and the same involution on the
//    ds_read_b128 address, which makes every 16-lane read group conflict-free;
//  * waves are 4 (rows) x 2 (column halves), 64 x BN/2 each; the MFMA operands
//    are swapped (A operand = weight fragment) so a lane's 4 accumulator
//    registers are 4 consecutive output columns of one row: 8-byte bf16
//    stores, and LayerNorm reduces over lanes {r, r+16, r+32, r+48} plus one
//    4 KB LDS exchange between the two column-half waves.
#include "common.hpp"

namespace {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef const __attribute__((address_space(1))) void* gbl_vptr;

constexpr int kThreads = 512;
constexpr int BM = 256;       // rows per block
constexpr int BK = 32;        // k per stage
constexpr int ROWB = BK * 2;  // bytes per staged row (64)
constexpr int NST = 4;        // stages in the ring

enum { BIG_LN = 0, BIG_ROWSCALE = 1 };

struct BigArgs {
  const uint16_t* a0; int64_t lda0; int k0;   // A columns [0, k0)
  const uint16_t* a1; int64_t lda1;           // A columns [k0, K)
  int K;
  const uint16_t* b; int64_t ldb;             // B [Nc][K] (weights)
  int64_t M; int Nc; int bn; int grid_y;
  uint16_t* out; int64_t ldo;
  uint16_t* xhat; float* rstd;
  const float* bias; const float* gamma; const float* beta;
  float eps, slope, drop_p, drop_scale; sldm::Seed seed; int64_t row_off;
  const int32_t* rowptr; int scale_cols;
  uint16_t* out2; int64_t ldo2;               // optional home of columns >= scale_cols
};

__device__ __forceinline__ void dma16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_vptr)g, (lds_vptr)lds_base, 16, 0, 0);
}

__device__ __forceinline__ int swz(int r16) { return (r16 >> 2) & 2; }

template <int NT, int MODE>
__global__ __launch_bounds__(kThreads, 2) void gemm_big_kernel(BigArgs p) {
  constexpr int BN = NT * 32;                  // columns per block
  constexpr int IPW = (BM + BN) / 16 / 8;      // DMA instructions per wave per stage
  constexpr int STAGE = (BM + BN) * ROWB;      // bytes per stage
  static_assert((BM + BN) % 128 == 0, "uniform DMA count per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem + NST * STAGE);   // [2 passes][BM][2]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
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
  if (m0 >= p.M) return;                       // XCD-mapping padding (whole block)
  const int n0 = cb * BN;

  // ---- DMA issue of one k-slice into a stage buffer ------------------------
  // Wave w fills 16-row groups w + 8j of the [A rows | B rows] image; lane l
  // lands at +16*l = row (l>>2), slot (l&3), which holds k-chunk slot^swz(row).
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ swz(drow);
  auto issue = [&](int buf, int kk) {
    char* base = smem + buf * STAGE;
    const uint16_t* abase;
    int64_t lda;
    int kc;
    if (kk < p.k0) { abase = p.a0; lda = p.lda0; kc = kk; }
    else           { abase = p.a1; lda = p.lda1; kc = kk - p.k0; }
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      const int g = wave + 8 * j;               // 16-row group in the image
      if (g < BM / 16) {
        const int64_t row = min(m0 + g * 16 + drow, p.M - 1);
        dma16(abase + row * lda + kc + 8 * dchunk, base + g * 16 * ROWB);
      } else {
        const int gc = g - BM / 16;
        const int col = min(n0 + gc * 16 + drow, p.Nc - 1);
        dma16(p.b + (int64_t)col * p.ldb + kk + 8 * dchunk, base + g * 16 * ROWB);
      }
    }
  };

  f4v acc[4][NT];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[m][t] = f4v{0.f, 0.f, 0.f, 0.f};

  const int nks = p.K / BK;
  // Prologue: stages 0 .. NST-2 in flight.
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s, min(s, nks - 1) * BK);

  const int roff = 16 * (q ^ swz(r16));          // byte offset of this lane's chunk
  for (int ks = 0; ks < nks; ++ks) {
    // Stage ks has landed for this wave once at most the (NST-2) younger
    // stages' DMAs are outstanding; the barrier extends that to all waves and
    // also retires every read of the buffer refilled just below.
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * IPW) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    {
      // Refill the buffer read in iteration ks-1 with slice ks+NST-1 (clamped:
      // past the end it re-reads the last slice, keeping the count uniform).
      const int kn = min(ks + NST - 1, nks - 1);
      issue((ks + NST - 1) % NST, kn * BK);
    }
    const char* cur = smem + (ks % NST) * STAGE;
    s8v af[4], bf[NT];
#pragma unroll
    for (int m = 0; m < 4; ++m)
      af[m] = *reinterpret_cast<const s8v*>(cur + (64 * wm + 16 * m + r16) * ROWB + roff);
#pragma unroll
    for (int t = 0; t < NT; ++t)
      bf[t] = *reinterpret_cast<const s8v*>(cur + (BM + wn * NT * 16 + 16 * t + r16) * ROWB + roff);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int t = 0; t < NT; ++t)
        acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[t], af[m], acc[m][t], 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the clamped tail DMAs

  // ---- epilogue -------------------------------------------------------------
  // acc[m][t][r] = C[row m0 + 64wm + 16m + r16][col n0 + wn*BN/2 + 16t + 4q + r]
  const int cbase = wn * (BN / 2) + 4 * q;        // + 16t: first of 4 columns (block-local)
  if constexpr (MODE == BIG_LN) {
    float bvec[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = cbase + 16 * t;
#pragma unroll
      for (int r = 0; r < 4; ++r) bvec[t][r] = p.bias ? p.bias[c + r] : 0.f;
    }
    const float inv_n = 1.0f / (float)p.Nc;
    const uint32_t dthr = sldm::dropout_threshold(p.drop_p);
    float mean[4], rstdv[4];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      float part[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        float s = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[m][t][r] + bvec[t][r];
            if (pass == 0) s += v;
            else { const float d = v - mean[m]; s += d * d; }
          }
        // lanes r16, r16+16, r16+32, r16+48 hold the same row
        s += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(s), 0x401F));
        s += __shfl_xor(s, 32, 64);
        part[m] = s;
      }
      if (q == 0) {
#pragma unroll
        for (int m = 0; m < 4; ++m) red[(pass * BM + 64 * wm + 16 * m + r16) * 2 + wn] = part[m];
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float* rr = red + (pass * BM + 64 * wm + 16 * m + r16) * 2;
        const float tot = rr[0] + rr[1];
        if (pass == 0) mean[m] = tot * inv_n;
        else rstdv[m] = 1.0f / sqrtf(tot * inv_n + p.eps);
      }
    }
    float gv[NT][4], bv[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gv[t][r] = p.gamma[cbase + 16 * t + r];
        bv[t][r] = p.beta[cbase + 16 * t + r];
      }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t row = m0 + 64 * wm + 16 * m + r16;
      if (row >= p.M) continue;
      if (p.rstd && q == 0 && wn == 0) p.rstd[row] = rstdv[m];
      const uint32_t rkey = sldm::dropout_row_key(sldm::effective_seed(p.seed), (uint64_t)(row + p.row_off));
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int c = cbase + 16 * t;
        float xh[4], z[4];
        bool keep[4] = {true, true, true, true};
        if (p.drop_p > 0.f) {
          sldm::dropout_keep2(rkey, (uint32_t)c, dthr, keep[0], keep[1]);
          sldm::dropout_keep2(rkey, (uint32_t)c + 2, dthr, keep[2], keep[3]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          xh[r] = (acc[m][t][r] + bvec[t][r] - mean[m]) * rstdv[m];
          const float y = xh[r] * gv[t][r] + bv[t][r];
          const float a = y > 0.f ? y : y * p.slope;
          z[r] = keep[r] ? a * p.drop_scale : 0.f;
        }
        sldm::Vec<uint16_t, 4>::store(p.out + row * p.ldo + c, z);
        if (p.xhat) sldm::Vec<uint16_t, 4>::store(p.xhat + row * p.ldo + c, xh);
      }
    }
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t row = m0 + 64 * wm + 16 * m + r16;
      if (row >= p.M) continue;
      float cnt = 1.f;
      if (p.rowptr) {
        const int deg = p.rowptr[row + 1] - p.rowptr[row];
        cnt = (float)(deg > 0 ? deg : 1);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int c = n0 + cbase + 16 * t;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[m][t][r];
          if (c + r < p.scale_cols) v[r] = v[r] / cnt;
        }
        if (c < p.Nc) {
          uint16_t* dst = p.out2 && c >= p.scale_cols ? p.out2 + row * p.ldo2 + (c - p.scale_cols)
                                                      : p.out + row * p.ldo + c;
          sldm::Vec<uint16_t, 4>::store(dst, v);
        }
      }
    }
  }
}

template <int NT, int MODE>
int launch_big(BigArgs& p, hipStream_t stream) {
  constexpr int BN = NT * 32;
  constexpr size_t lds = (size_t)NST * (BM + BN) * ROWB + 2 * BM * 2 * sizeof(float);
  int64_t nrb = (p.M + BM - 1) / BM;
  if (p.grid_y > 1) nrb = (nrb + 7) / 8 * 8;
  const int64_t grid = nrb * p.grid_y;
  SLDM_REQUIRE(grid < ((int64_t)1 << 31), "gemm_big: grid too large");
  auto kern = gemm_big_kernel<NT, MODE>;
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, kThreads, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("gemm_big_kernel");
  return SLDM_OK;
}

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

}  // namespace

namespace sldm {

bool big_gemm_enabled() {
  static const bool on = [] {
    const char* e = getenv("SLDM_BIG_GEMM");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Shape gate shared by the dispatchers in gemm.hip: bf16, K and the A split
// multiples of the 32-deep k-slice, BN of 128 or 256, 16-byte aligned rows.
bool big_gemm_ok(int64_t k0, int64_t K, int64_t bn, const void* a0, int64_t lda0,
                 const void* a1, int64_t lda1, const void* b, int64_t ldb, int64_t ldo) {
  if (K % BK || k0 % BK || (bn != 128 && bn != 256)) return false;
  if (lda0 % 8 || (K > k0 && lda1 % 8) || ldb % 8 || ldo % 4) return false;
  return aligned16(a0) && (K == k0 || aligned16(a1)) && aligned16(b);
}

int big_dense_fwd(const void* a0, int64_t lda0, int64_t k0, const void* a1, int64_t lda1,
                  int64_t k1, const void* w, int64_t num_rows, int64_t nc, const float* bias,
                  const float* gamma, const float* beta, float eps, float slope, float drop_p,
                  uint64_t seed, int64_t row_off, void* out, void* xhat, float* rstd,
                  hipStream_t stream) {
  BigArgs p{};
  p.a0 = (const uint16_t*)a0; p.lda0 = lda0; p.k0 = (int)k0;
  p.a1 = k1 ? (const uint16_t*)a1 : (const uint16_t*)a0; p.lda1 = k1 ? lda1 : lda0;
  p.K = (int)(k0 + k1);
  p.b = (const uint16_t*)w; p.ldb = k0 + k1;
  p.M = num_rows; p.Nc = (int)nc; p.bn = (int)nc; p.grid_y = 1;
  p.out = (uint16_t*)out; p.ldo = nc; p.xhat = (uint16_t*)xhat; p.rstd = rstd;
  p.bias = bias; p.gamma = gamma; p.beta = beta; p.eps = eps; p.slope = slope;
  p.drop_p = drop_p;
  p.drop_scale = drop_p >= 1.f ? 0.f : (drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f);
  p.seed = seed; p.row_off = row_off;
  return nc == 256 ? launch_big<8, BIG_LN>(p, stream) : launch_big<4, BIG_LN>(p, stream);
}

int big_gemm_rowscale(const void* a, int64_t lda, int64_t k, const void* b, int64_t ldb,
                      int64_t num_rows, int64_t nc, int64_t bn, const int32_t* rowptr,
                      int64_t scale_cols, void* out, int64_t ldo, void* out2, int64_t ldo2,
                      hipStream_t stream) {
  BigArgs p{};
  p.a0 = (const uint16_t*)a; p.lda0 = lda; p.k0 = (int)k;
  p.a1 = (const uint16_t*)a; p.lda1 = lda;
  p.K = (int)k;
  p.b = (const uint16_t*)b; p.ldb = ldb;
  p.M = num_rows; p.Nc = (int)nc; p.bn = (int)bn;
  p.grid_y = (int)((nc + bn - 1) / bn);
  p.out = (uint16_t*)out; p.ldo = ldo;
  p.out2 = (uint16_t*)out2; p.ldo2 = ldo2;
  p.rowptr = rowptr; p.scale_cols = (int)scale_cols;
  return bn == 256 ? launch_big<8, BIG_ROWSCALE>(p, stream)
                   : launch_big<4, BIG_ROWSCALE>(p, stream);
}

}  // namespace sldm
