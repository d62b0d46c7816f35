// Persistent fp32 kernels for the dense part of a SageBlock layer at
// F_out = 256: the forward (bias + LayerNorm + activation + dropout epilogue)
// and the 1/deg-prescaled dX GEMM, on six-term split-bf16 products
// (sldm::split3_bf16x4 / SLDM_MFMA_X6 in common.hpp: fp32-level results from
// the bf16 MFMA).
//
// The 64-row tile kernel (gemm.hip, gemm_nt_x6_kernel) stages every A tile with
// a load -> split -> LDS -> barrier -> compute sequence and re-reads and
// re-splits its fp32 weight fragments in every wave and k-step: its MFMAs idle
// through both.  At six MFMAs per product the GEMM is MFMA-bound (15.7 TFLOP
// per launch at 10M rows = 6.3 ms at the dense bf16 peak against 5-6.5 ms of
// HBM time), so this kernel is built to keep the matrix pipe fed:
//
//  * one 512-thread workgroup per CU loops over 256-row tiles; wave w owns
//    rows [32w, 32w + 32) x all 256 output columns (128 accumulator VGPRs), so
//    LayerNorm statistics reduce in-wave and a weight fragment read from LDS
//    feeds 12 MFMAs;
//  * activations never touch LDS: each lane loads its MFMA operand's fp32
//    values straight from HBM about a k-step ahead (a k-step is ~2.5 us of
//    MFMA work per SIMD; the sequence runs on across tile boundaries, so the
//    next tile's first loads are in flight under the epilogue) and splits
//    them into hi / mid / lo fragments in registers (~56 VALU per k-step
//    against 192 MFMAs);
//  * none of that work stands between the barrier and the MFMAs: loads,
//    splits and LDS writes are placed between the step's MFMA groups, where
//    they issue while the matrix pipe runs;
//  * the 32-deep weight slice of a k-step is fetched from L2 as fp32 half a
//    step ahead by all waves together (each wave 32 columns), split once, and
//    written as three bf16 images into a 2-stage LDS ring: one barrier per
//    k-step, 48 KB per stage;
//  * within a k-step lane q of a fragment holds k = {4q..4q+3, 16+4q..16+4q+3}
//    (both operands alike; the contraction does not care), so every activation
//    load instruction reads 16 rows x 64 contiguous bytes;
//  * 512 output columns (dX = dZ [W_l | W_r]) run as two column halves on
//    workgroup pairs of one XCD (blocks b and b + 8), which walk the same row
//    tiles at the same time: the second read of a tile hits that XCD's L2.
//
// Every vector-memory op is a plain load or store: the compiler counts vmcnt.
// The k-step barrier is a raw s_barrier behind an LDS-only wait, so the
// prefetched global loads stay in flight across it.
#include "common.hpp"

namespace {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;
constexpr int NW = 8;             // waves per workgroup
constexpr int RW = 32;            // rows per wave
constexpr int BM = NW * RW;       // rows per tile
constexpr int NTT = 16;           // 16-column MFMA tiles per wave (256 columns)
constexpr int IMG = 256 * 64;     // bytes of one bf16 image of a 32-deep slice of 256 weight rows
constexpr int WSTAGE = 3 * IMG;   // hi | mid | lo

enum { SF_LN = 0, SF_ROWSCALE = 1 };
// Diagnostic builds only (tools/ab_build.sh; results wrong, timing only):
// 1 = no MFMAs, 6 = no split arithmetic (raw bits as fragments), 8 = no
// activation reloads, 9 = no weight reloads, 10 = no output stores.
#ifndef SLDM_SF_EXP
#define SLDM_SF_EXP 0
#endif

struct SfArgs {
  const float* a0; int64_t lda0;       // A columns [0, K) or [0, K/2) when SPLIT
  const float* a1; int64_t lda1;       // A columns [K/2, K) when SPLIT
  const float* b; int64_t ldb;         // weights [halves * 256][K]
  int64_t M; int64_t ntiles; int halves;
  float* out; int64_t ldo;
  float* xhat; float* rstd;
  const float* bias; const float* gamma; const float* beta;
  float eps, slope, drop_p, drop_scale; sldm::Seed seed; int64_t row_off;
  const int32_t* rowptr; int scale_cols;
  float* out2; int64_t ldo2;           // ROWSCALE: optional home of columns >= scale_cols
};

// 16-B chunk swizzle of a 64-B weight row (conflict-free fragment reads; the
// image layout of gemm_stream.hip / gemm_big.hip)
__device__ __forceinline__ int swz(int r16) { return (r16 >> 2) & 2; }

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int KSTEPS, int MODE, bool SPLIT, bool HASDEG>
__global__ __launch_bounds__(kThreads) void gemm_stream_x6_kernel(SfArgs p) {
  static_assert(KSTEPS % 2 == 0 && KSTEPS >= 4, "ring shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wring = smem;                                              // 2 stages x 3 images
  float* prm = reinterpret_cast<float*>(smem + 2 * WSTAGE);        // bias | gamma | beta

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // (tile, column half) of this workgroup: pairs b, b + 8 share an XCD
  int half = 0;
  int64_t tile, tstride;
  if (p.halves == 2) {
    const int b = blockIdx.x, xcd = b & 7, j = b >> 3;
    half = j & 1;
    tile = (int64_t)(j >> 1) * 8 + xcd;
    tstride = gridDim.x >> 1;
  } else {
    tile = blockIdx.x;
    tstride = gridDim.x;
  }
  if (tile >= p.ntiles) return;
  const float* wb = p.b + (int64_t)half * 256 * p.ldb;

  if constexpr (MODE == SF_LN) {
    for (int i = tid; i < 256; i += kThreads) {
      prm[i] = p.bias ? p.bias[i] : 0.f;
      prm[256 + i] = p.gamma[i];
      prm[512 + i] = p.beta[i];
    }
  }

  // Every per-lane address below is rebuilt inside its k-step from a lane id
  // the compiler cannot see through (volatile v_mbcnt pair, no inputs): with
  // visible lane ids the 16 unrolled k-steps' address tables are hoisted out
  // of the tile loop and spill beside the 128 accumulators.  Uniform parts
  // stay on scalar bases; k offsets are immediates.
  auto lane_id = []() {
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    return ln;
  };
  // ---- weight slice: wave w stages columns [32w, 32w + 32); lane -> column
  // 8i + (lane >> 3) of them in load i, floats [4 piece, 4 piece + 4) of the
  // slice (whole 128-B lines per 8 lanes) ----
  auto load_w1 = [&](int ks, int i, f4v& w, int ln) {
    const uint32_t woff =
        (uint32_t)((wave * 32 + (ln >> 3)) * (uint32_t)p.ldb + 4 * (ln & 7)) * 4u;
    const char* sl = reinterpret_cast<const char*>(wb) + 128 * ks;
    w = *reinterpret_cast<const f4v*>(sl + (size_t)(32 * i) * (size_t)p.ldb + woff);
  };
  auto store_w1 = [&](int slot, int i, const f4v& w, int ln) {
    char* base = wring + slot * WSTAGE;
    const int piece = ln & 7;
    const int c = wave * 32 + (ln >> 3) + 8 * i;
    const float f[4] = {w[0], w[1], w[2], w[3]};
    uint2 h, md, l;
#if SLDM_SF_EXP == 6      // diagnostic: no split arithmetic (raw bits stored)
    h = make_uint2(__float_as_uint(f[0]), __float_as_uint(f[1]));
    md = make_uint2(__float_as_uint(f[2]), __float_as_uint(f[3]));
    l = h;
#else
    sldm::split3_bf16x4(f, h, md, l);
#endif
    // floats 4 piece.. of the slice are elements 4 (piece >> 2).. of chunk piece & 3
    const int off = c * 64 + 16 * ((piece & 3) ^ swz(c & 15)) + 8 * (piece >> 2);
    *reinterpret_cast<uint2*>(base + off) = h;
    *reinterpret_cast<uint2*>(base + IMG + off) = md;
    *reinterpret_cast<uint2*>(base + 2 * IMG + off) = l;
  };
  // ---- activation fragments: lane (r16, q) <- row r16 (+16m), floats
  // [4q, 4q + 4) and [16 + 4q, 16 + 4q + 4) of the k-step; rows past M clamp.
  // One 32-bit row offset serves both operands (host-checked: lda1 == lda0) ----
  auto load_a = [&](int64_t tl, int ks, f4v (&dst)[2][2], int ln) {
    const int kk = ks * 32;
    const bool h = SPLIT && kk >= KSTEPS * 16;
    const int64_t r0 = tl * BM;
    const char* base = reinterpret_cast<const char*>(
        (h ? p.a1 + (kk - KSTEPS * 16) : p.a0 + kk) + r0 * p.lda0);
    const int last = (int)min<int64_t>(p.M - 1 - r0, BM - 1);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int rr = min(wave * RW + 16 * m + (ln & 15), last);
      const uint32_t voff = ((uint32_t)rr * (uint32_t)p.lda0 + 4 * (ln >> 4)) * 4u;
      dst[m][0] = *reinterpret_cast<const f4v*>(base + voff);
      dst[m][1] = *reinterpret_cast<const f4v*>(base + voff + 64);
    }
  };
  struct Frag { s8v h, m, l; };
  auto split_a = [&](const f4v (&raw)[2], Frag& fr) {
    const float f[8] = {raw[0][0], raw[0][1], raw[0][2], raw[0][3],
                        raw[1][0], raw[1][1], raw[1][2], raw[1][3]};
#if SLDM_SF_EXP == 6
    fr.h = __builtin_bit_cast(s8v, make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]),
                                              __float_as_uint(f[2]), __float_as_uint(f[3])));
    fr.m = __builtin_bit_cast(s8v, make_uint4(__float_as_uint(f[4]), __float_as_uint(f[5]),
                                              __float_as_uint(f[6]), __float_as_uint(f[7])));
    fr.l = fr.h;
#else
    sldm::split3_bf16x8(f, fr.h, fr.m, fr.l);
#endif
  };

  f4v araw[2][2];      // [m][half of the fragment]: raw values of the k-step after next
  f4v wraw[2];         // raw weight values: two of the next slice's four pieces at a time
  Frag af[2];          // this k-step's activation fragments
  f4v acc[2][NTT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < NTT; ++t) acc[m][t] = f4v{0.f, 0.f, 0.f, 0.f};

  {
    const int ln = lane_id();
    load_a(tile, 0, araw, ln);
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      load_w1(0, 2 * h2, wraw[0], ln);
      load_w1(0, 2 * h2 + 1, wraw[1], ln);
      store_w1(0, 2 * h2, wraw[0], ln);
      store_w1(0, 2 * h2 + 1, wraw[1], ln);
    }
    load_w1(1, 0, wraw[0], ln);
    load_w1(1, 1, wraw[1], ln);
    split_a(araw[0], af[0]);
    split_a(araw[1], af[1]);
    load_a(tile, 1, araw, ln);
  }

  for (;;) {
    const int64_t nraw = tile + tstride;
    const bool has_next = nraw < p.ntiles;
    const int64_t next = has_next ? nraw : tile;   // tail: harmless re-load

    int dg[2][2] = {{0, 1}, {0, 1}};
    if constexpr (HASDEG) {
      const int ln = lane_id();
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int64_t row = min(tile * BM + wave * RW + 16 * m + (ln & 15), p.M - 1);
        dg[m][0] = p.rowptr[row];
        dg[m][1] = p.rowptr[row + 1];
      }
    }

    // A k-step: one barrier, then 16 column tiles of 12 MFMAs; the step's
    // other work rides between them in program order (a full scheduling
    // barrier per column tile keeps it there): the next slice's four weight
    // pieces are split into the other LDS stage two at a time, half a step
    // after their loads (tiles 0, 2 and 8, 10); behind the last tile's MFMAs
    // the next step's activation values -- loaded a step ago -- are split into
    // the fragment registers and reloaded for the step after next.  Weight
    // fragments are read one column tile ahead, in a scheduling region of
    // their own (left free, the reads sink to just before their use).
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      // slice ks is complete in stage ks & 1 and every wave is done reading
      // the other stage (its reads fed the previous step's MFMAs)
      lds_barrier();
      const int ln = lane_id();
      const char* cur =
          wring + (ks & 1) * WSTAGE + (ln & 15) * 64 + 16 * ((ln >> 4) ^ swz(ln & 15));
      s8v wf[2][3];
      auto read_w = [&](int t, s8v (&w)[3]) {
#pragma unroll
        for (int i = 0; i < 3; ++i) w[i] = *reinterpret_cast<const s8v*>(cur + t * 1024 + i * IMG);
      };
      read_w(0, wf[0]);
#pragma unroll
      for (int t = 0; t < NTT; ++t) {
        if (t + 1 < NTT) read_w(t + 1, wf[(t + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#if SLDM_SF_EXP == 1      // diagnostic: no MFMAs (operands kept alive)
        asm volatile("" ::"v"(wf[t & 1][0]), "v"(wf[t & 1][1]), "v"(wf[t & 1][2]));
        asm volatile("" ::"v"(af[0].h), "v"(af[0].m), "v"(af[0].l));
        asm volatile("" ::"v"(af[1].h), "v"(af[1].m), "v"(af[1].l));
#else
#pragma unroll
        for (int m = 0; m < 2; ++m)
          SLDM_MFMA_X6(acc[m][t], wf[t & 1][0], wf[t & 1][1], wf[t & 1][2], af[m].h, af[m].m,
                       af[m].l);
#endif
        if (t == 0 || t == 2 || t == 8 || t == 10) {
          // slice ks + 1 (the next tile's past the end): pieces 0, 1 now, their
          // registers reloaded with pieces 2, 3, which go half a step later
          const int r = (t >> 1) & 1, pc = (t >= 8 ? 2 : 0) + r;
          store_w1((ks + 1) & 1, pc, wraw[r], ln);
#if SLDM_SF_EXP != 9      // diagnostic 9: no weight reloads (timing only)
          if (t < 8) load_w1((ks + 1) % KSTEPS, pc + 2, wraw[r], ln);
          else load_w1((ks + 2) % KSTEPS, pc - 2, wraw[r], ln);
#else
          asm volatile("" : "+v"(wraw[r]));
#endif
        }
        if (t == NTT - 1) {
          // after the step's last MFMAs have issued: their operands' registers
          // take the next step's fragments while the matrix pipe drains (the
          // scheduling barrier keeps the new values from overlapping the old)
          __builtin_amdgcn_sched_barrier(0);
          split_a(araw[0], af[0]);
          split_a(araw[1], af[1]);
#if SLDM_SF_EXP != 8      // diagnostic 8: no activation reloads (timing only)
          if (ks + 2 < KSTEPS) load_a(tile, ks + 2, araw, ln);
          else load_a(next, ks + 2 - KSTEPS, araw, ln);
#else
          asm volatile("" : "+v"(araw[0][0]), "+v"(araw[0][1]), "+v"(araw[1][0]), "+v"(araw[1][1]));
#endif
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }

#if SLDM_SF_EXP == 10    // diagnostic 10: no output stores (timing only)
#define SF_STORE(ptr, v) do { if (p.eps < 0.f) *reinterpret_cast<f4v*>(ptr) = (v); } while (0)
#else
#define SF_STORE(ptr, v) (*reinterpret_cast<f4v*>(ptr) = (v))
#endif
    const int q = lane_id() >> 4, r16 = lane_id() & 15;
    // ---- epilogue: acc[m][t][r] = C[row 16m + r16][col 16t + 4q + r] ----
    if constexpr (MODE == SF_LN) {
      const float inv_n = 1.0f / 256.f;
      const uint32_t dthr = sldm::dropout_threshold(p.drop_p);
      const int cq = 4 * q;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        // rows past M (final tile only) hold row M-1's values (clamped loads):
        // clamping the row everywhere (dropout key included) makes their
        // stores identical rewrites of row M-1
        const int64_t row = min(tile * BM + wave * RW + 16 * m + r16, p.M - 1);
        float s = 0.f;
#pragma unroll
        for (int t = 0; t < NTT; ++t) {
          const f4v bb = *reinterpret_cast<const f4v*>(prm + 16 * t + cq);
          acc[m][t] += bb;
#pragma unroll
          for (int r = 0; r < 4; ++r) s += acc[m][t][r];
        }
        s = sldm::row4_sum(s);
        const float mean = s * inv_n;
        float v2 = 0.f;
#pragma unroll
        for (int t = 0; t < NTT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = acc[m][t][r] - mean;
            acc[m][t][r] = d;
            v2 += d * d;
          }
        v2 = sldm::row4_sum(v2);
        const float rs = 1.0f / sqrtf(v2 * inv_n + p.eps);
        if (p.rstd && q == 0) p.rstd[row] = rs;
        const uint32_t rkey = sldm::dropout_row_key(sldm::effective_seed(p.seed), (uint64_t)(row + p.row_off));
        float* xrow = p.xhat ? p.xhat + row * p.ldo + cq : nullptr;
        float* orow = p.out + row * p.ldo + cq;
#pragma unroll
        for (int t = 0; t < NTT; ++t) {
          const int c = 16 * t + cq;
          const f4v xh = acc[m][t] * rs;
          if (xrow) SF_STORE(xrow + 16 * t, xh);
          const f4v gg = *reinterpret_cast<const f4v*>(prm + 256 + c);
          const f4v be = *reinterpret_cast<const f4v*>(prm + 512 + c);
          bool keep[4] = {true, true, true, true};
          if (p.drop_p > 0.f) {
            sldm::dropout_keep2(rkey, (uint32_t)c, dthr, keep[0], keep[1]);
            sldm::dropout_keep2(rkey, (uint32_t)c + 2, dthr, keep[2], keep[3]);
          }
          f4v o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float y = __builtin_fmaf(xh[r], gg[r], be[r]);   // as post_bwd recomputes it
            const float a = y > 0.f ? y : y * p.slope;
            o[r] = keep[r] ? a * p.drop_scale : 0.f;
          }
          SF_STORE(orow + 16 * t, o);
        }
      }
    } else {
      // a half's 256 columns all go to one buffer (host-checked: scale_cols a
      // multiple of 256 when out2 is set)
      float* obase = p.out;
      int64_t ldo = p.ldo;
      const int c0 = half * 256;
      if (p.out2 && c0 >= p.scale_cols) { obase = p.out2 - p.scale_cols; ldo = p.ldo2; }
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int64_t row = min(tile * BM + wave * RW + 16 * m + r16, p.M - 1);
        const int deg = dg[m][1] - dg[m][0];
        const float cnt = (float)(deg > 0 ? deg : 1);   // divided, as the tile kernels do
        float* orow = obase + row * ldo + c0 + 4 * q;
#pragma unroll
        for (int t = 0; t < NTT; ++t) {
          // scale_cols is a multiple of 16: one uniform test per tile
          const bool scaled = HASDEG && c0 + 16 * t < p.scale_cols;
          f4v o = acc[m][t];
          if (scaled) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = o[r] / cnt;
          }
          SF_STORE(orow + 16 * t, o);
        }
      }
    }
#undef SF_STORE

    if (!has_next) break;
    tile = next;
#pragma unroll
    for (int i = 0; i < 2 * NTT; ++i) acc[i / NTT][i % NTT] = f4v{0.f, 0.f, 0.f, 0.f};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // retire the tail's unused prefetches
}

int g_num_cus = 0;
int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    g_num_cus = n;
  }
  return g_num_cus;
}

template <int KSTEPS, int MODE, bool SPLIT, bool HASDEG = false>
int launch_sf(SfArgs& p, hipStream_t stream) {
  constexpr size_t lds = 2 * WSTAGE + 3 * 256 * sizeof(float);
  static_assert(lds <= 160 * 1024, "LDS budget");
  p.ntiles = (p.M + BM - 1) / BM;
  int64_t grid;
  if (p.halves == 2) {
    // tile slots in multiples of 8 (one per XCD), two workgroups per slot
    const int64_t max_slots = std::max<int64_t>(8, (num_cus() / 2) / 8 * 8);
    const int64_t slots = std::min<int64_t>((p.ntiles + 7) / 8 * 8, max_slots);
    grid = 2 * slots;
  } else {
    grid = std::min<int64_t>(p.ntiles, num_cus());
  }
  auto kern = gemm_stream_x6_kernel<KSTEPS, MODE, SPLIT, HASDEG>;
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, kThreads, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("gemm_stream_x6_kernel");
  return SLDM_OK;
}

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

}  // namespace

namespace sldm {

// Read per call so tests can pin the stream and tile kernels to each other.
bool stream_f32_enabled() {
  const char* e = getenv("SLDM_STREAM_F32");
  return !(e && e[0] == '0');
}

// Shape gate of the fp32 stream kernels: K of 256 or 512 (one operand, or two
// of K/2 each), rows and bases 16-byte aligned.
static bool stream_f32_common_ok(int64_t k0, int64_t K, const void* a0, int64_t lda0,
                                 const void* a1, int64_t lda1, const void* b, int64_t ldb) {
  if ((K != 256 && K != 512) || (k0 != K && 2 * k0 != K)) return false;
  if (k0 != K && lda1 != lda0) return false;   // one row offset serves both operands
  if (lda0 % 4 || ldb % 4 || lda0 > (1 << 20) || ldb > (1 << 20)) return false;
  return aligned16(a0) && (K == k0 || aligned16(a1)) && aligned16(b);
}

bool stream_f32_dense_fwd_ok(int64_t k0, int64_t K, int64_t nc, const void* a0, int64_t lda0,
                             const void* a1, int64_t lda1, const void* w, const void* out,
                             const void* xhat) {
  return nc == 256 && stream_f32_common_ok(k0, K, a0, lda0, a1, lda1, w, K) && aligned16(out) &&
         (!xhat || aligned16(xhat));
}

bool stream_f32_rowscale_ok(int64_t k, int64_t nc, const void* a, int64_t lda, const void* b,
                            int64_t ldb, const void* out, int64_t ldo, const void* out2,
                            int64_t ldo2, int64_t scale_cols) {
  if ((nc != 256 && nc != 512) || ldo % 4 || scale_cols % 16) return false;
  if (out2 && (ldo2 % 4 || !aligned16(out2) || scale_cols % 256)) return false;
  return stream_f32_common_ok(k, k, a, lda, a, lda, b, ldb) && aligned16(out);
}

int stream_f32_dense_fwd(const void* a0, int64_t lda0, int64_t k0, const void* a1, int64_t lda1,
                         int64_t k1, const void* w, int64_t num_rows, const float* bias,
                         const float* gamma, const float* beta, float eps, float slope,
                         float drop_p, uint64_t seed, int64_t row_off, void* out, void* xhat,
                         float* rstd, hipStream_t stream) {
  SfArgs p{};
  p.a0 = (const float*)a0; p.lda0 = lda0;
  p.a1 = k1 ? (const float*)a1 : (const float*)a0; p.lda1 = k1 ? lda1 : lda0;
  const int K = (int)(k0 + k1);
  p.b = (const float*)w; p.ldb = K;
  p.M = num_rows; p.halves = 1;
  p.out = (float*)out; p.ldo = 256; p.xhat = (float*)xhat; p.rstd = rstd;
  p.bias = bias; p.gamma = gamma; p.beta = beta; p.eps = eps; p.slope = slope;
  p.drop_p = drop_p;
  p.drop_scale = drop_p >= 1.f ? 0.f : (drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f);
  p.seed = seed; p.row_off = row_off;
  if (k1 == 0)
    return K == 512 ? launch_sf<16, SF_LN, false>(p, stream) : launch_sf<8, SF_LN, false>(p, stream);
  return K == 512 ? launch_sf<16, SF_LN, true>(p, stream) : launch_sf<8, SF_LN, true>(p, stream);
}

int stream_f32_gemm_rowscale(const void* a, int64_t lda, int64_t k, const void* b, int64_t ldb,
                             int64_t num_rows, int64_t nc, const int32_t* rowptr,
                             int64_t scale_cols, void* out, int64_t ldo, void* out2, int64_t ldo2,
                             hipStream_t stream) {
  SfArgs p{};
  p.a0 = (const float*)a; p.lda0 = lda;
  p.a1 = (const float*)a; p.lda1 = lda;
  p.b = (const float*)b; p.ldb = ldb;
  p.M = num_rows; p.halves = (int)(nc / 256);
  p.out = (float*)out; p.ldo = ldo;
  p.out2 = (float*)out2; p.ldo2 = ldo2;
  p.rowptr = rowptr; p.scale_cols = (int)scale_cols;
  if (rowptr)
    return k == 512 ? launch_sf<16, SF_ROWSCALE, false, true>(p, stream)
                    : launch_sf<8, SF_ROWSCALE, false, true>(p, stream);
  return k == 512 ? launch_sf<16, SF_ROWSCALE, false, false>(p, stream)
                  : launch_sf<8, SF_ROWSCALE, false, false>(p, stream);
}

}  // namespace sldm
