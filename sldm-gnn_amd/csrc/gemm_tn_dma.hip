// Weight-gradient GEMM of the SageBlock backward at F = 256, bf16:
//   dW[256][n0 + n1] = dZ^T @ [agg | h]      (sum over the node rows)
// as a row-streaming kernel: each workgroup owns one 256 x 256 output half
// (columns of agg, or of h) over a contiguous chunk of node rows, so every
// input row is read once per half (dZ twice -- both halves of a chunk run on
// one XCD at the same time, the second read an L2 hit) instead of once per
// 128 x 128 tile as in gemm.hip's gemm_tn_kernel (4x dZ, 2x agg/h through the
// CU load path; 33 % LDS bank-conflict cycles in its padded tiles:
// profiles/r1c_stall_pmc.json).
//
//  * 512 threads, 8 waves as 2 (m) x 4 (n): 128 x 64 outputs per wave, 128
//    fp32 accumulators per lane;
//  * k-steps of 32 node rows: dZ [32][256] and B [32][256] (16 KB each) arrive
//    by LDS-DMA (1 KB contiguous per instruction) in a ring of NBUF slots,
//    one counted `s_waitcnt vmcnt` + s_barrier per k-step;
//  * MFMA operands need 8 consecutive ROWS per lane: ds_read_b64_tr_b16 on a
//    32-B-granule XOR swizzle (granule g of row r at g ^ f(r), f(r) = (r & 3)
//    | ((r & 8) >> 1)) that puts the 8 rows of each 32-lane transpose group on
//    8 distinct 32-B bank groups -- conflict-free;
//  * partial sums per chunk go to a [splits][256][nn] fp32 slab, reduced in
//    split order by gemm.hip's slab_reduce_kernel (deterministic).
#include "common.hpp"

namespace {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vptr;

constexpr int kThreads = 512;
constexpr int kKRows = 32;                  // node rows per k-step
constexpr int kSub = kKRows * 512;          // one operand's k-step tile (16 KB)
constexpr int kNbuf = 4;

struct Tn2Args {
  const uint16_t* a; int64_t lda;           // dZ [rows][256]
  const uint16_t* b0; int64_t ldb0;         // [rows][256] -> output columns [0, 256)
  const uint16_t* b1; int64_t ldb1;         // [rows][256] -> output columns [256, 512)
  int64_t rows, chunk;                      // chunk: rows per split (multiple of 32)
  int splits, halves, nn;
  float* slab;                              // [splits][256][nn]
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void dma16(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
}
__device__ __forceinline__ int swz(int r) { return (r & 3) | ((r & 8) >> 1); }

__global__ __launch_bounds__(kThreads) void gemm_tn_dma_kernel(Tn2Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // blockIdx -> (split, half): both halves of a split share blockIdx % 8 (one
  // XCD under round-robin dispatch) and launch together
  const int b = blockIdx.x;
  const int half = p.halves == 2 ? (b >> 3) & 1 : 0;
  const int split = p.halves == 2 ? ((b >> 4) << 3) + (b & 7) : b;
  const int64_t kbeg = (int64_t)split * p.chunk;
  const int64_t kend = min(kbeg + p.chunk, p.rows);
  const int64_t nks = kend > kbeg ? (kend - kbeg + kKRows - 1) / kKRows : 0;
  const uint16_t* bsrc = half ? p.b1 : p.b0;
  const int64_t ldb = half ? p.ldb1 : p.ldb0;

  // ---- DMA of k-step ks into slot ks % kNbuf: waves 0-3 dZ, 4-7 B, 4 each
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_vptr)smem;
  auto issue = [&](int64_t ks) {
    // tail slots re-load the last k-step; an empty split loads rows [0, 32)
    const int64_t k0 = nks > 0 ? kbeg + (ks < nks ? ks : nks - 1) * kKRows : 0;
    const int64_t last = p.rows - 1 - k0;   // rows past the end clamp (masked in the MFMA)
    const bool isb = wave >= 4;
    const char* base = reinterpret_cast<const char*>(isb ? bsrc + k0 * ldb : p.a + k0 * p.lda);
    const int64_t ld = isb ? ldb : p.lda;
    uint32_t la = lds0 + (uint32_t)((ks % kNbuf) * 2 * kSub + (isb ? kSub : 0));
    asm volatile("" : "+s"(base), "+s"(la));
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = (wave & 3) * 4 + j;               // instruction in the sub-tile
      const int gp = d * 64 + ln;                     // 16-B granule in the sub-tile
      const int r = gp >> 5, p16 = gp & 31;
      const int g32 = (p16 >> 1) ^ swz(r);            // logical 32-B granule
      const int64_t rr = r < last ? r : last;
      const uint32_t voff = (uint32_t)(rr * ld * 2 + 32 * g32 + 16 * (p16 & 1));
      dma16(base, voff, la + (uint32_t)(d * 1024));
    }
  };

  f4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < kNbuf - 1; ++s) issue(s);

  for (int64_t ks = 0; ks < nks; ++ks) {
    wait_vm<(kNbuf - 2) * 4>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(ks + kNbuf - 1);

    int q, r16;
    {
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      q = ln >> 4;
      r16 = ln & 15;
    }
    const char* sa = smem + (ks % kNbuf) * 2 * kSub;
    const char* sb = sa + kSub;
    // lane (q, r16) addresses row 8q + (r16 >> 2) (+4 for the high half),
    // byte 8 (r16 & 3) of its column tile's 32-B granule; it receives column
    // r16 of rows 8q .. 8q+7 (the MFMA operand of a 32-deep k-step)
    const int rlo = 8 * q + (r16 >> 2), rhi = rlo + 4;
    const int cb = 8 * (r16 & 3);
    auto tr = [&](const char* sub, int r, int g32) {
      return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s4v*)(sub + r * 512 + 32 * (g32 ^ swz(r)) + cb));
    };
    // node rows past the chunk end (clamped duplicates) contribute nothing:
    // both operands zeroed, so a duplicated Inf cannot turn into NaN
    const bool partial = kbeg + (ks + 1) * kKRows > kend;   // uniform
    const int64_t krow = kbeg + ks * kKRows + 8 * q;        // this lane's first k row
    auto mask = [&](s8v& v) {
      if (partial) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (krow + e >= kend) v[e] = 0;
      }
    };
    s8v bf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // one 16-column MFMA tile = one 32-B granule
      const int g32 = (wn * 64 + 16 * j) >> 4;
      const s4v lo = tr(sb, rlo, g32), hi = tr(sb, rhi, g32);
      bf[j] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      mask(bf[j]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int g32 = (wm * 128 + 16 * i) >> 4;
      const s4v lo = tr(sa, rlo, g32), hi = tr(sa, rhi, g32);
      s8v af = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      mask(af);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[j], acc[i][j], 0, 0, 0);
    }
  }
  wait_vm<0>();

  // partial tile -> slab[split]: acc[i][j][r] = dW[m = 128 wm + 16 i + 4 q + r]
  //                                               [n = 256 half + 64 wn + 16 j + r16]
  const int q = lane >> 4, r16 = lane & 15;
  float* out = p.slab + (int64_t)split * 256 * p.nn + 256 * half;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(int64_t)(wm * 128 + 16 * i + 4 * q + r) * p.nn + wn * 64 + 16 * j + r16] =
            acc[i][j][r];
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

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

}  // namespace

namespace sldm {

bool tn_dma_enabled() {
  const char* e = getenv("SLDM_TN_DMA");
  return !(e && e[0] == '0');
}

// Split plan: one workgroup per CU (halves x splits = CU count), each split
// at least 8 k-steps; splits a multiple of 8 when halves == 2 (XCD pairing).
static void tn_dma_plan(int64_t rows, int halves, int& splits, int64_t& chunk) {
  int64_t s = num_cus() / halves;
  const int64_t max_s = (rows + 8 * kKRows - 1) / (8 * kKRows);
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  if (halves == 2 && s >= 8) s = s / 8 * 8;
  if (halves == 2 && s < 8) s = 8;   // keeps the blockIdx mapping a bijection (empty splits write 0)
  chunk = (rows + s - 1) / s;
  chunk = (chunk + kKRows - 1) / kKRows * kKRows;
  splits = (int)s;
}

bool tn_dma_ok(int64_t mo, int64_t n0, int64_t n1, int64_t rows, const void* a, int64_t lda,
               const void* b0, int64_t ldb0, const void* b1, int64_t ldb1) {
  if (mo != 256 || n0 != 256 || (n1 != 0 && n1 != 256) || rows >= (int64_t(1) << 31)) return false;
  if (lda % 8 || ldb0 % 8 || lda > (1 << 20) || ldb0 > (1 << 20)) return false;
  if (n1 && (ldb1 % 8 || ldb1 > (1 << 20) || !aligned16(b1))) return false;
  return aligned16(a) && aligned16(b0);
}

size_t tn_dma_workspace_bytes(int64_t rows, int64_t nn) {
  int splits;
  int64_t chunk;
  tn_dma_plan(rows, nn == 512 ? 2 : 1, splits, chunk);
  return sizeof(float) * (size_t)splits * 256 * (size_t)nn + 256;
}

// Runs the kernel into `slab` and returns the split count (the caller reduces).
int tn_dma(const void* a, int64_t lda, const void* b0, int64_t ldb0, const void* b1, int64_t ldb1,
           int64_t n1, int64_t rows, float* slab, int* splits_out, hipStream_t stream) {
  Tn2Args p{};
  p.a = (const uint16_t*)a; p.lda = lda;
  p.b0 = (const uint16_t*)b0; p.ldb0 = ldb0;
  p.b1 = n1 ? (const uint16_t*)b1 : (const uint16_t*)b0; p.ldb1 = n1 ? ldb1 : ldb0;
  p.rows = rows;
  p.halves = n1 ? 2 : 1;
  p.nn = n1 ? 512 : 256;
  tn_dma_plan(rows, p.halves, p.splits, p.chunk);
  p.slab = slab;
  constexpr size_t lds = (size_t)kNbuf * 2 * kSub;
  static_assert(lds <= 160 * 1024, "LDS budget");
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_tn_dma_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  gemm_tn_dma_kernel<<<(unsigned)(p.splits * p.halves), kThreads, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("gemm_tn_dma_kernel");
  *splits_out = p.splits;
  return SLDM_OK;
}

}  // namespace sldm
