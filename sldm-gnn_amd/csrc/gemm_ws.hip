// Weight-stationary bf16 MFMA kernel for the dX GEMM of the SageBlock backward:
//   out[:, :scale_cols] = (dZ @ W^T)[:, :scale_cols] / deg     (dAgg)
//   out2 / out[:, scale_cols:] = (dZ @ W^T)[:, scale_cols:]   (root-branch dH)
// with W = [W_l | W_r]^T stored [Nc][K] (Nc = 512, K = 256 at F = 256).
//
// Why not the stream kernel (gemm_stream.hip): there every k-step re-streams a
// 32-deep slice of all Nc weight rows from L2 into LDS, i.e. |W| = 256 KB per
// 128-row tile = 2 KB of L2 traffic per output row on top of the 1.5 KB of
// HBM traffic -- the per-CU vector-memory path (TA, 78 % busy, stalled on the
// TCP's pending misses: profiles/r1c_stall_pmc.json) is the bound, not HBM.
// Here the weights never move after the prologue:
//
//  * wave w of the 512-thread workgroup holds output columns
//    [16*CT*w, 16*CT*(w+1)) x all K of W in VGPRs (CT*KSTEPS MFMA A-fragments,
//    128 VGPRs at Nc = 512, K = 256), loaded once;
//  * activation tiles of TM rows (32 KB) stream HBM -> LDS by LDS-DMA in a
//    ring of NBUF slots, each DMA instruction reading 1 KB contiguous (whole
//    rows) and writing a row-XOR-swizzled image (granule j of row r at
//    j ^ (r & 15)) so the MFMA B-fragment reads (ds_read_b128, lane = row i,
//    16-B k-chunk q) are bank-conflict-free in every ds_read_b128 lane group;
//  * one counted `s_waitcnt vmcnt` + s_barrier per TILE (not per k-step);
//    NBUF-1 tiles are in flight while a tile computes and its epilogue stores;
//  * the epilogue is gemm_stream.hip's: 1/deg row scale, tiles paired through
//    v_permlane16_swap into one 16-B store per lane.
// The MFMA sequence per output element (k-steps in order, same instruction)
// is the stream kernel's, so results are bit-identical to it.
//
// vmcnt bookkeeping (per wave, every op opaque asm or a plain store): per tile
// the wave issues DPW activation DMAs (+1 rowptr DMA) for tile n+NBUF-1, then
// RG*CT/2 epilogue stores for tile n.  At the top of tile n >= NBUF-1 the ops
// younger than tile n's DMAs are ST + (NBUF-2)*(DMA+ST); before that only the
// prologue's (NBUF-2)*DMA are guaranteed younger (a stricter count).
#include "common.hpp"

namespace {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vptr;

constexpr int kThreads = 512;
constexpr int kTileBytes = 32768;   // activation bytes per tile
constexpr int kRpBytes = 8 * 256;   // per-wave rowptr DMA landing zones

struct WsArgs {
  const uint16_t* a; int64_t lda;     // activations [M][K]
  const uint16_t* b; int64_t ldb;     // weights [Nc][K]
  int64_t M; int64_t ntiles;
  uint16_t* out; int64_t ldo;
  uint16_t* out2; int64_t ldo2;       // optional home of columns >= scale_cols
  const int32_t* rowptr; int scale_cols;
  int blk_shift;                      // > 0: ``out`` is [scale_cols >> blk_shift][M][1 << blk_shift]
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// 64 lanes x 16 B from sbase + voff[lane] to LDS [m0, m0 + 1 KB), lane-linear.
__device__ __forceinline__ void dma16(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
}
// 64 lanes x 4 B, lane-linear into [m0, m0 + 256).
__device__ __forceinline__ void dma4(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1"
               :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
}

template <int KSTEPS, int NBUF, bool HASDEG>
constexpr size_t ws_lds_bytes() {
  return (size_t)NBUF * (kTileBytes + (HASDEG ? kRpBytes : 0));
}

template <int KSTEPS, int CT, int NBUF, bool HASDEG>
__global__ __launch_bounds__(kThreads) void ws_rowscale_kernel(WsArgs p) {
  constexpr int RB = KSTEPS * 64;              // bytes per activation row (K * 2)
  constexpr int G = RB / 16;                   // 16-B granules per row
  constexpr int TM = kTileBytes / RB;          // rows per tile
  constexpr int RG = TM / 16;                  // 16-row MFMA groups per tile
  constexpr int DPW = kTileBytes / 1024 / 8;   // activation DMAs per wave per tile
  constexpr int RPW = TM / 8;                  // rows per wave's rowptr zone
  constexpr int SLOT = kTileBytes + (HASDEG ? kRpBytes : 0);
  constexpr int OPS_DMA = DPW + (HASDEG ? 1 : 0);
  constexpr int OPS_ST = RG * CT / 2;
  constexpr int VM_STEADY = OPS_ST + (NBUF - 2) * (OPS_DMA + OPS_ST);
  constexpr int VM_START = (NBUF - 2) * OPS_DMA;
  static_assert(G >= 16 && TM % 16 == 0 && CT % 2 == 0 && NBUF >= 2, "tile shape");
  static_assert(VM_STEADY <= 63, "vmcnt range");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  if ((int64_t)blockIdx.x >= p.ntiles) return;
  const int64_t grid = gridDim.x;

  // ---- weights: this wave's CT column tiles x KSTEPS k-steps, in VGPRs ----
  const int cbase = wave * 16 * CT;
  s8v wf[CT][KSTEPS];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
      wf[ct][s] = *reinterpret_cast<const s8v*>(
          p.b + (int64_t)(cbase + 16 * ct + (lane & 15)) * p.ldb + 32 * s + 8 * (lane >> 4));

  // ---- DMA issue for the block's n-th tile into slot n % NBUF ----
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_vptr)smem;
  auto tile_of = [&](int64_t n) -> int64_t {
    const int64_t t = blockIdx.x + n * grid;
    return t < p.ntiles ? t : (int64_t)blockIdx.x;   // tail: harmless re-load
  };
  auto issue = [&](int64_t n) {
    const int64_t r0 = tile_of(n) * TM;
    const char* base = reinterpret_cast<const char*>(p.a + r0 * p.lda);
    const int64_t last = p.M - 1 - r0;   // >= 0: rows past M clamp to M-1
    uint32_t la = lds0 + (uint32_t)((n % NBUF) * SLOT);
    asm volatile("" : "+s"(base), "+s"(la));
    // lane id re-derived here (volatile, no inputs) so no per-lane offset
    // table is hoisted out of the tile loop and kept live beside the weights
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const int gp = (wave * DPW + j) * 64 + ln;     // LDS granule in the tile
      const int r = gp / G, jg = gp % G;
      const int64_t rr = r < last ? r : last;
      const uint32_t voff = (uint32_t)(rr * p.lda * 2 + 16 * (jg ^ (r & 15)));
      dma16(base, voff, la + (uint32_t)((wave * DPW + j) * 1024));
    }
    if constexpr (HASDEG) {
      const int64_t e = r0 + RPW * wave + ln;
      const uint32_t voff = (uint32_t)((e < p.M ? e : p.M) * 4);
      dma4(p.rowptr, voff, la + kTileBytes + wave * 256);
    }
  };

#pragma unroll
  for (int n = 0; n < NBUF - 1; ++n) issue(n);

  // scale/out routing is uniform per wave (host-checked: scale_cols % (16*CT) == 0)
  const bool scaled = HASDEG && cbase < p.scale_cols;
  uint16_t* obase = p.out;
  int64_t ldo = p.ldo;
  if (p.out2 && cbase >= p.scale_cols) { obase = p.out2 - p.scale_cols; ldo = p.ldo2; }
  // column-blocked home of the scaled half (the send layout of a feature-
  // sliced partition's all-to-all): block c >> sh holds columns [c, c + 2^sh)
  // of every row, contiguous; a lane's 8 columns never straddle a block
  const int sh = p.blk_shift;
  const bool blocked = sh > 0 && cbase < p.scale_cols;

  for (int64_t n = 0;; ++n) {
    const int64_t tile = blockIdx.x + n * grid;
    if (tile >= p.ntiles) break;
    // lane-derived values re-derived per tile (nothing per-lane tile-invariant
    // for LICM to keep live beside the 128 weight VGPRs)
    int i, q;
    {
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      i = ln & 15;
      q = ln >> 4;
    }
    const int ccol = cbase + ((q & 1) ? 16 + 4 * (q - 1) : 4 * q);
    if (n < NBUF - 1) wait_vm<VM_START>();
    else wait_vm<VM_STEADY>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(n + NBUF - 1);

    const char* slot = smem + (n % NBUF) * SLOT;
    f4v acc[RG][CT];
#pragma unroll
    for (int m = 0; m < RG; ++m)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[m][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    // B fragments one k-step ahead: step s's MFMAs run while step s+1's
    // ds_reads are in flight (pinned below, so at most 2*RG fragments live)
    s8v bf[2][RG];
    auto read_b = [&](int s, s8v (&dst)[RG]) {
      const int goff = 16 * ((4 * s + q) ^ i);
#pragma unroll
      for (int m = 0; m < RG; ++m)
        dst[m] = *reinterpret_cast<const s8v*>(slot + (16 * m + i) * RB + goff);
    };
    read_b(0, bf[0]);
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      if (s + 1 < KSTEPS) read_b(s + 1, bf[(s + 1) & 1]);
#pragma unroll
      for (int m = 0; m < RG; ++m)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
          acc[m][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ct][s], bf[s & 1][m], acc[m][ct],
                                                              0, 0, 0);
      if (s + 1 < KSTEPS) __builtin_amdgcn_sched_group_barrier(0x100, RG, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, RG * CT, 0);
    }

    // ---- epilogue: acc[m][ct][r] = C[row 16m + i][col cbase + 16ct + 4q + r]
    const int64_t r0 = tile * TM;
#pragma unroll
    for (int m = 0; m < RG; ++m) {
      // rows past M hold row M-1's (clamped) activations and rewrite row M-1:
      // clamp the degree's row too, or those rewrites would carry deg 1
      const int tr = 16 * m + i < p.M - 1 - r0 ? 16 * m + i : (int)(p.M - 1 - r0);
      const int64_t row = r0 + tr;
      float inv = 1.f;
      if (scaled) {
        const int32_t* rp =
            reinterpret_cast<const int32_t*>(slot + kTileBytes + (tr / RPW) * 256) + tr % RPW;
        const int deg = rp[1] - rp[0];
        inv = 1.0f / (float)(deg > 0 ? deg : 1);
      }
#pragma unroll
      for (int t = 0; t < CT; t += 2) {
        uint32_t w[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = scaled ? acc[m][t + h][r] * inv : acc[m][t + h][r];
          w[h][0] = sldm::pack_bf16x2(v[0], v[1]);
          w[h][1] = sldm::pack_bf16x2(v[2], v[3]);
        }
        auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
        auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
        uint16_t* dst = obase + row * ldo + ccol + 16 * t;
        if (blocked) {
          const int c = ccol + 16 * t;
          dst = p.out + ((((int64_t)(c >> sh)) * p.M + row) << sh) + (c & ((1 << sh) - 1));
        }
        *reinterpret_cast<uint4*>(dst) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    }
  }
  wait_vm<0>();   // retire the tail's dummy DMAs before the workgroup ends
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

template <int KSTEPS, int CT, int NBUF, bool HASDEG>
int launch_ws(WsArgs& p, hipStream_t stream) {
  constexpr int TM = kTileBytes / (KSTEPS * 64);
  constexpr size_t lds = ws_lds_bytes<KSTEPS, NBUF, HASDEG>();
  static_assert(lds <= 160 * 1024, "LDS budget");
  p.ntiles = (p.M + TM - 1) / TM;
  const int64_t grid = std::min<int64_t>(p.ntiles, num_cus());
  auto kern = ws_rowscale_kernel<KSTEPS, CT, NBUF, HASDEG>;
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, kThreads, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("ws_rowscale_kernel");
  return SLDM_OK;
}

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

}  // namespace

namespace sldm {

// Read per call (not cached) so tests can pin both dX kernels to each other.
bool ws_gemm_enabled() {
  const char* e = getenv("SLDM_WS_GEMM");
  return !(e && e[0] == '0');
}
// Shape gate: bf16 (caller), K = 256, Nc = 512 (CT = 4) or 256 (CT = 2),
// 16-B aligned rows and bases; a split / scaled boundary on a wave's column
// block; row stride and count small enough for 32-bit DMA offsets.
bool ws_rowscale_ok(int64_t k, int64_t nc, int64_t num_rows, const void* a, int64_t lda,
                    const void* b, int64_t ldb, const void* out, int64_t ldo, const void* out2,
                    int64_t ldo2, int64_t scale_cols) {
  if (k != 256 || (nc != 512 && nc != 256) || num_rows >= (int64_t(1) << 30)) return false;
  const int64_t wcols = nc / 8;
  if (scale_cols % wcols || lda % 8 || ldb % 8 || ldo % 8 || lda > (1 << 20)) return false;
  if (out2 && (ldo2 % 8 || !aligned16(out2))) return false;
  return aligned16(a) && aligned16(b) && aligned16(out);
}

int ws_gemm_rowscale(const void* a, int64_t lda, int64_t k, const void* b, int64_t ldb,
                     int64_t num_rows, int64_t nc, const int32_t* rowptr, int64_t scale_cols,
                     void* out, int64_t ldo, void* out2, int64_t ldo2, hipStream_t stream,
                     int blk_shift) {
  (void)k;
  WsArgs p{};
  p.blk_shift = blk_shift;
  p.a = (const uint16_t*)a; p.lda = lda;
  p.b = (const uint16_t*)b; p.ldb = ldb;
  p.M = num_rows;
  p.out = (uint16_t*)out; p.ldo = ldo;
  p.out2 = (uint16_t*)out2; p.ldo2 = ldo2;
  p.rowptr = rowptr; p.scale_cols = (int)scale_cols;
  if (nc == 512)
    return rowptr ? launch_ws<8, 4, 4, true>(p, stream) : launch_ws<8, 4, 4, false>(p, stream);
  return rowptr ? launch_ws<8, 2, 4, true>(p, stream) : launch_ws<8, 2, 4, false>(p, stream);
}

}  // namespace sldm
