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
        *reinterpret_cast<uint4*>(obase + row * ldo + ccol + 16 * t) =
            make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    }
  }
  wait_vm<0>();   // retire the tail's dummy DMAs before the workgroup ends
}

// ---------------------------------------------------------------------------
// Forward dense layer, same weight-stationary scheme, LayerNorm epilogue:
//   z = [a0 | a1] @ W^T + bias  (W [256][K], K = k0 + k1),
//   xhat = (z - mean) * rstd, out = dropout(act(xhat * gamma + beta)).
// Wave w holds output columns [32w, 32w + 32) (CT = 2 tiles) x all K of W
// (KSTEPS*8 VGPRs: 128 at K = 512).  A tile slot holds two LDS sub-tiles,
// [TM][k0] from a0 then [TM][k1] from a1, each row-XOR-swizzled; every DMA
// instruction lands in one sub-tile, so its 64 lanes share one SGPR base.
// The MFMA layout spreads each row's 256 columns over the 8 waves; the
// epilogue re-distributes z through LDS so that one wave owns whole rows
// (epilogue comment).
struct WsLnArgs {
  const uint16_t* a0; int64_t lda0;
  const uint16_t* a1; int64_t lda1;
  const uint16_t* w;                  // [256][K]
  int64_t M; int64_t ntiles;
  uint16_t* out; uint16_t* xhat; float* rstd;   // [M][256], [M][256], [M]
  const float* bias; const float* gamma; const float* beta;
  float eps, slope, drop_p, drop_scale; uint64_t seed; int64_t row_off;
};

// XCHG selects the epilogue: false re-distributes z through LDS so one wave
// owns whole rows ([TM][256] fp32 staging); true keeps z in the MFMA layout and
// exchanges only the per-row LayerNorm partial sums (2 x [TM][8] fp32).
#ifndef SLDM_WSLN_PF
#define SLDM_WSLN_PF 2
#endif
constexpr int WSLN_PF = SLDM_WSLN_PF;
// Diagnostic builds only (tools/ab_build.sh): 1 = the exchange kernel with a
// plain store epilogue, 2 = without its MFMAs; the pipelined kernel 3 = without
// the row-sum exchange and its barrier, 4 = with a plain pack-and-store
// output stage.  Results are wrong in all four.
#ifndef SLDM_WSLN_EXP
#define SLDM_WSLN_EXP 0
#endif

template <int KSTEPS, int NBUF, int TM, bool XCHG>
constexpr size_t ws_ln_lds_bytes() {
  return (size_t)NBUF * TM * KSTEPS * 64 + 3 * 256 * sizeof(float) +
         (XCHG ? (size_t)2 * TM * 8 * sizeof(float) : (size_t)TM * 1024);
}

template <int KSTEPS, int K0STEPS, int NBUF, int TM, bool XCHG>
__global__ __launch_bounds__(kThreads) void ws_ln_kernel(WsLnArgs p) {
  constexpr int CT = 2;
  constexpr int K1STEPS = KSTEPS - K0STEPS;
  constexpr int RB0 = K0STEPS * 64, RB1 = K1STEPS * 64;   // sub-tile row bytes
  constexpr int TB = TM * KSTEPS * 64;                    // tile bytes (16 or 32 KB)
  constexpr int RG = TM / 16;
  constexpr int DPW = TB / 1024 / 8;
  constexpr int SUB1 = TM * RB0;                          // byte offset of sub-tile 1
  constexpr int OPS_DMA = DPW;
  static_assert(K0STEPS % 4 == 0 && K1STEPS % 4 == 0 && SUB1 % 1024 == 0, "sub-tile shape");
  static_assert(TB % 8192 == 0 && NBUF >= 2, "tile shape");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* prm = reinterpret_cast<float*>(smem + NBUF * TB);   // bias | gamma | beta
  char* zs = reinterpret_cast<char*>(prm + 3 * 256);          // [TM][256] fp32 z, swizzled
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  if ((int64_t)blockIdx.x >= p.ntiles) return;
  const int64_t grid = gridDim.x;

  for (int c = tid; c < 256; c += kThreads) {
    prm[c] = p.bias ? p.bias[c] : 0.f;
    prm[256 + c] = p.gamma[c];
    prm[512 + c] = p.beta[c];
  }

  const int cbase = wave * 16 * CT;
  const int64_t K = KSTEPS * 32;
  s8v wf[CT][KSTEPS];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
      wf[ct][s] = *reinterpret_cast<const s8v*>(
          p.w + (int64_t)(cbase + 16 * ct + (lane & 15)) * K + 32 * s + 8 * (lane >> 4));

  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_vptr)smem;
  auto tile_of = [&](int64_t n) -> int64_t {
    const int64_t t = blockIdx.x + n * grid;
    return t < p.ntiles ? t : (int64_t)blockIdx.x;
  };
  // Per-lane DMA offsets of a full tile, computed once (tile-invariant); a
  // final partial tile recomputes them with its rows clamped to M-1.
  uint32_t voff0[DPW];
  auto dma_off = [&](int j, int64_t last) -> uint32_t {
    const int d = wave * DPW + j;
    const bool sub1 = d * 1024 >= SUB1;
    const int ob = sub1 ? d * 1024 - SUB1 : d * 1024;
    const int gsub = (sub1 ? RB1 : RB0) / 16;
    const int gp = ob / 16 + lane;
    const int r = gp / gsub, jg = gp % gsub;
    const int64_t rr = r < last ? r : last;
    return (uint32_t)(rr * (sub1 ? p.lda1 : p.lda0) * 2 + 16 * (jg ^ (r & 15)));
  };
#pragma unroll
  for (int j = 0; j < DPW; ++j) voff0[j] = dma_off(j, TM);
  auto issue = [&](int64_t n) {
    const int64_t r0 = tile_of(n) * TM;
    const int64_t last = p.M - 1 - r0;
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const int d = wave * DPW + j;                 // wave-uniform
      const bool sub1 = d * 1024 >= SUB1;
      const char* base = reinterpret_cast<const char*>(sub1 ? p.a1 + r0 * p.lda1
                                                            : p.a0 + r0 * p.lda0);
      uint32_t la = lds0 + (uint32_t)((n % NBUF) * TB + d * 1024);
      asm volatile("" : "+s"(base), "+s"(la));
      dma16(base, last >= TM - 1 ? voff0[j] : dma_off(j, last), la);
    }
  };

#pragma unroll
  for (int n = 0; n < NBUF - 1; ++n) issue(n);

  const float inv_n = 1.0f / 256.f;
  const uint32_t dthr = sldm::dropout_threshold(p.drop_p);
  const bool hasx = p.xhat != nullptr;
  const int nst = 2 + (hasx ? 2 : 0) + (p.rstd ? 1 : 0);

  for (int64_t n = 0;; ++n) {
    const int64_t tile = blockIdx.x + n * grid;
    if (tile >= p.ntiles) break;
    int i, q;
    {
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      i = ln & 15;
      q = ln >> 4;
    }
    // stores per wave per tile: 2 out (+ 2 xhat) (+ 1 rstd), the same in
    // every wave
    if (n < NBUF - 1) {
      wait_vm<(NBUF - 2) * OPS_DMA>();
    } else {
      switch (nst) {
        case 2: wait_vm<2 + (NBUF - 2) * (OPS_DMA + 2)>(); break;
        case 3: wait_vm<3 + (NBUF - 2) * (OPS_DMA + 3)>(); break;
        case 4: wait_vm<4 + (NBUF - 2) * (OPS_DMA + 4)>(); break;
        default: wait_vm<5 + (NBUF - 2) * (OPS_DMA + 5)>(); break;
      }
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(n + NBUF - 1);

    f4v acc[RG][CT];
#pragma unroll
    for (int m = 0; m < RG; ++m)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[m][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    // B-fragment addresses: (4 ls + q) ^ i = 4 (ls ^ (i >> 2)) + ((q ^ i) & 3)
    // for ls = 4a + b, so a lane's address is one of 4 per-lane values (b)
    // plus compile-time offsets (a, m, sub-tile) -- no per-read VALU.
    typedef __attribute__((address_space(3))) const s8v* lds_frag;
    const uint32_t sl = lds0 + (uint32_t)((n % NBUF) * TB);
    uint32_t lb0[4], lb1[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t o = (uint32_t)(64 * (b ^ (i >> 2)) + 16 * ((q ^ i) & 3));
      lb0[b] = sl + (uint32_t)(i * RB0) + o;
      lb1[b] = sl + (uint32_t)(SUB1 + i * RB1) + o;
    }
    // B fragments PF k-steps ahead (PF = 1 for the z-redistributing epilogue)
    constexpr int PF = XCHG ? WSLN_PF : 1;
    s8v bf[PF + 1][RG];
    auto read_b = [&](int s, s8v (&dst)[RG]) {
      const bool s1 = s >= K0STEPS;
      const int ls = s1 ? s - K0STEPS : s;
      const int rb = s1 ? RB1 : RB0;
      const uint32_t a = (s1 ? lb1 : lb0)[ls & 3] + (uint32_t)(256 * (ls >> 2));
#pragma unroll
      for (int m = 0; m < RG; ++m) dst[m] = *(lds_frag)(uintptr_t)(a + (uint32_t)(16 * m * rb));
    };
#pragma unroll
    for (int s = 0; s < PF; ++s) read_b(s, bf[s]);
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      if (s + PF < KSTEPS) read_b(s + PF, bf[(s + PF) % (PF + 1)]);
#pragma unroll
      for (int m = 0; m < RG; ++m)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#if SLDM_WSLN_EXP == 2
          acc[m][ct] += __builtin_bit_cast(f4v, __builtin_shufflevector(bf[s % (PF + 1)][m],
                                                                        bf[s % (PF + 1)][m], 0, 1, 2, 3, 4, 5, 6, 7));
#else
          acc[m][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ct][s], bf[s % (PF + 1)][m],
                                                              acc[m][ct], 0, 0, 0);
#endif
      if (s + PF < KSTEPS) __builtin_amdgcn_sched_group_barrier(0x100, RG, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, RG * CT, 0);
    }

#if SLDM_WSLN_EXP == 1
    if constexpr (XCHG) {   // experiment: main loop + plain bf16 stores of z
      const int64_t r0 = tile * TM;
      const int ccol = cbase + ((q & 1) ? 16 + 4 * (q - 1) : 4 * q);
#pragma unroll
      for (int m = 0; m < RG; ++m) {
        const int64_t row = r0 + 16 * m + i < p.M ? r0 + 16 * m + i : p.M - 1;
        uint32_t w[2][2];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          w[ct][0] = sldm::pack_bf16x2(acc[m][ct][0], acc[m][ct][1]);
          w[ct][1] = sldm::pack_bf16x2(acc[m][ct][2], acc[m][ct][3]);
        }
        auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
        auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
        const uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        if (hasx) *reinterpret_cast<uint4*>(p.xhat + row * 256 + ccol) = v;
        *reinterpret_cast<uint4*>(p.out + row * 256 + ccol) = v;
      }
      if (p.rstd && lane < 32) p.rstd[r0 + lane < p.M ? r0 + lane : p.M - 1] = 1.f;
      continue;
    }
#endif
    if constexpr (XCHG) {
      // ---- epilogue, exchange form: acc[m][ct][r] = z[row 16m + i][col
      // cbase + 16ct + 4q + r] stays in place.  Row sums: in-lane over the
      // lane's 8 columns, then over the 4 lanes of the row (q, xor 16 / 32),
      // then the 8 waves' partials through LDS (red[row][wave], summed in wave
      // order after a barrier); the same for the squared deviations.  Two
      // buffers, so tile n+1's first exchange never races tile n's reads (every
      // wave has read buffer 0 before it reaches the second barrier).
      float* red = reinterpret_cast<float*>(zs);
      float tot[RG];
      auto row_total = [&](float (&part)[RG], int buf, float (&sum)[RG]) {
#pragma unroll
        for (int m = 0; m < RG; ++m) {
          const float v = sldm::row4_sum(part[m]);
          if (q == 0) red[(buf * TM + 16 * m + i) * 8 + wave] = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int m = 0; m < RG; ++m) {
          const f4v* pr = reinterpret_cast<const f4v*>(red + (buf * TM + 16 * m + i) * 8);
          const f4v a = pr[0], b = pr[1];
          sum[m] = a[0] + a[1] + a[2] + a[3] + b[0] + b[1] + b[2] + b[3];
        }
      };
      float part[RG];
#pragma unroll
      for (int m = 0; m < RG; ++m) {
        part[m] = 0.f;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const f4v bb = *reinterpret_cast<const f4v*>(prm + cbase + 16 * ct + 4 * q);
          acc[m][ct] += bb;
#pragma unroll
          for (int r = 0; r < 4; ++r) part[m] += acc[m][ct][r];
        }
      }
      row_total(part, 0, tot);
#pragma unroll
      for (int m = 0; m < RG; ++m) {
        const float mean = tot[m] * inv_n;
        part[m] = 0.f;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = acc[m][ct][r] - mean;
            acc[m][ct][r] = d;
            part[m] += d * d;
          }
      }
      row_total(part, 1, tot);
      const int64_t r0 = tile * TM;
      const int ccol = cbase + ((q & 1) ? 16 + 4 * (q - 1) : 4 * q);
      float rs[RG];
#pragma unroll
      for (int m = 0; m < RG; ++m) {
        rs[m] = 1.0f / sqrtf(tot[m] * inv_n + p.eps);
        // rows past M hold row M-1's (clamped) activations and rewrite row M-1
        const int64_t row = r0 + 16 * m + i < p.M ? r0 + 16 * m + i : p.M - 1;
        const uint32_t rkey = sldm::dropout_row_key(p.seed, (uint64_t)(row + p.row_off));
        uint32_t wx[CT][2], wo[CT][2];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
          const int c = cbase + 16 * ct + 4 * q;
          const f4v gg = *reinterpret_cast<const f4v*>(prm + 256 + c);
          const f4v be = *reinterpret_cast<const f4v*>(prm + 512 + c);
          bool keep[4] = {true, true, true, true};
          if (p.drop_p > 0.f) {
            sldm::dropout_keep2(rkey, (uint32_t)c, dthr, keep[0], keep[1]);
            sldm::dropout_keep2(rkey, (uint32_t)c + 2, dthr, keep[2], keep[3]);
          }
          float xh[4], o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            xh[r] = acc[m][ct][r] * rs[m];
            const float y = xh[r] * gg[r] + be[r];
            const float a = y > 0.f ? y : y * p.slope;
            o[r] = keep[r] ? a * p.drop_scale : 0.f;
          }
          wx[ct][0] = sldm::pack_bf16x2(xh[0], xh[1]);
          wx[ct][1] = sldm::pack_bf16x2(xh[2], xh[3]);
          wo[ct][0] = sldm::pack_bf16x2(o[0], o[1]);
          wo[ct][1] = sldm::pack_bf16x2(o[2], o[3]);
        }
        // tiles 0 and 1 leave together, one 16-B store per lane (ws_rowscale)
        if (hasx) {
          auto s0 = __builtin_amdgcn_permlane16_swap(wx[0][0], wx[1][0], false, false);
          auto s1 = __builtin_amdgcn_permlane16_swap(wx[0][1], wx[1][1], false, false);
          *reinterpret_cast<uint4*>(p.xhat + row * 256 + ccol) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
        auto s0 = __builtin_amdgcn_permlane16_swap(wo[0][0], wo[1][0], false, false);
        auto s1 = __builtin_amdgcn_permlane16_swap(wo[0][1], wo[1][1], false, false);
        *reinterpret_cast<uint4*>(p.out + row * 256 + ccol) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
      // rstd: one store per wave (the same count in every wave, for vmcnt):
      // lane l < 16 holds row l in rs[0], lane 16 + l row 16 + l in rs[1]
      if (p.rstd && lane < 32) {
        const int64_t row = r0 + lane < p.M ? r0 + lane : p.M - 1;
        p.rstd[row] = lane < 16 ? rs[0] : rs[1];
      }
      continue;
    }

    // ---- epilogue, row-owner form: the MFMA layout spreads a row over all 8
    // waves, so z goes to LDS (fp32, 16-B granule g of row r at g ^ (r & 7):
    // conflict-free for both the writes below and the reads after the
    // barrier) and wave w then owns tile rows 4w .. 4w+3 whole -- lane
    // (rr = lane >> 4, l = lane & 15) holds columns 8l + 128t + e (t < 2,
    // e < 8) of row 4w + rr, LayerNorm statistics reduce over its 16 lanes
    // (DPP), and each row leaves as 256-B contiguous 16-B-per-lane stores.
#pragma unroll
    for (int m = 0; m < RG; ++m)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int row = 16 * m + i, g = (cbase + 16 * ct + 4 * q) >> 2;
        *reinterpret_cast<f4v*>(zs + row * 1024 + 16 * (g ^ (row & 7))) = acc[m][ct];
      }
    __syncthreads();
    {
      const int rr = lane >> 4, l = lane & 15;
      const int trow = 4 * wave + rr;
      const int64_t r0 = tile * TM;
      // rows past M hold row M-1's values (clamped loads) and rewrite row M-1
      const int64_t row = r0 + trow < p.M ? r0 + trow : p.M - 1;
      float v[2][8];
      float sm = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int g = 2 * l + 32 * t + h;
          const f4v z = *reinterpret_cast<const f4v*>(zs + trow * 1024 + 16 * (g ^ (trow & 7)));
          const f4v bb = *reinterpret_cast<const f4v*>(prm + 4 * g);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[t][4 * h + e] = z[e] + bb[e];
            sm += v[t][4 * h + e];
          }
        }
      const float mean = sldm::group_sum(sm, 16) * inv_n;
      float v2 = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[t][e] -= mean;
          v2 += v[t][e] * v[t][e];
        }
      const float rs = 1.0f / sqrtf(sldm::group_sum(v2, 16) * inv_n + p.eps);
      if (p.rstd && l == 0) p.rstd[row] = rs;
      const uint32_t rkey = sldm::dropout_row_key(p.seed, (uint64_t)(row + p.row_off));
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int c0 = 8 * l + 128 * t;
        float xh[8], o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) xh[e] = v[t][e] * rs;
        if (hasx) sldm::Vec<uint16_t, 8>::store(p.xhat + row * 256 + c0, xh);
        bool keep[8] = {true, true, true, true, true, true, true, true};
        if (p.drop_p > 0.f) {
#pragma unroll
          for (int e = 0; e < 8; e += 2)
            sldm::dropout_keep2(rkey, (uint32_t)(c0 + e), dthr, keep[e], keep[e + 1]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float y = xh[e] * prm[256 + c0 + e] + prm[512 + c0 + e];
          const float a = y > 0.f ? y : y * p.slope;
          o[e] = keep[e] ? a * p.drop_scale : 0.f;
        }
        sldm::Vec<uint16_t, 8>::store(p.out + row * 256 + c0, o);
      }
    }
  }
  wait_vm<0>();
}

// ---------------------------------------------------------------------------
// Forward dense layer, weight-stationary, with the LayerNorm epilogue software-
// pipelined into the next tile's MFMA stream (SLDM_WS_FWD=3).  Same main loop
// and exchange statistics as ws_ln_kernel<XCHG>; the difference is where the
// epilogue's heavy half runs.  Per tile n:
//   top:   wait for tile n's A slice, barrier B0 (also publishes tile n-1's
//          squared-deviation partials), DMA of tile n+NBUF-1;
//   loop:  the 16 (8) k-steps of tile n's MFMAs, with tile n-1's output work
//          -- rstd, row keys, xhat, LN affine, activation, dropout hashes,
//          packing and stores -- placed between them in fixed pieces
//          (sched_barrier-pinned), so that VALU issues while the MFMAs run
//          instead of after them (at 2 lock-stepped waves per SIMD nothing
//          else overlaps them);
//   then:  bias + row sums of tile n -> LDS, barrier B1, mean, deviations
//          (kept in registers for the next iteration), squared sums -> LDS.
// Two barriers per tile instead of three; the last tile's output work runs
// after the loop.  vmcnt: per iteration the wave issues DPW DMAs, then the
// previous tile's NST stores, so the steady-state count is ws_ln_kernel's.
template <int KSTEPS, int K0STEPS, int NBUF, bool SAVE>
__global__ __launch_bounds__(kThreads) void ws_ln_pipe_kernel(WsLnArgs p) {
  constexpr int TM = 32, CT = 2, RG = 2;
  constexpr int K1STEPS = KSTEPS - K0STEPS;
  constexpr int RB0 = K0STEPS * 64, RB1 = K1STEPS * 64;
  constexpr int TB = TM * KSTEPS * 64;
  constexpr int DPW = TB / 1024 / 8;
  constexpr int SUB1 = TM * RB0;
  constexpr int NST = SAVE ? 5 : 2;                 // out 2 (+ xhat 2 + rstd 1)
  constexpr int VM_START = (NBUF - 2) * DPW;        // iterations n < NBUF
  constexpr int VM_STEADY = NST + (NBUF - 2) * (DPW + NST);
  constexpr int SLOT8 = KSTEPS / 8;                 // k-steps between epilogue pieces
  static_assert(K0STEPS % 4 == 0 && K1STEPS % 4 == 0 && SUB1 % 1024 == 0, "sub-tile shape");
  static_assert(TB % 8192 == 0 && NBUF >= 2 && KSTEPS % 8 == 0, "tile shape");
  static_assert(VM_STEADY <= 63, "vmcnt range");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* prm = reinterpret_cast<float*>(smem + NBUF * TB);   // bias | gamma | beta
  float* red = prm + 3 * 256;                                 // [2][TM][8]: sums | sq sums
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  if ((int64_t)blockIdx.x >= p.ntiles) return;
  const int64_t grid = gridDim.x;

  for (int c = tid; c < 256; c += kThreads) {
    prm[c] = p.bias ? p.bias[c] : 0.f;
    prm[256 + c] = p.gamma[c];
    prm[512 + c] = p.beta[c];
  }

  const int cbase = wave * 16 * CT;
  const int64_t K = KSTEPS * 32;
  s8v wf[CT][KSTEPS];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
      wf[ct][s] = *reinterpret_cast<const s8v*>(
          p.w + (int64_t)(cbase + 16 * ct + (lane & 15)) * K + 32 * s + 8 * (lane >> 4));

  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_vptr)smem;
  auto tile_of = [&](int64_t n) -> int64_t {
    const int64_t t = blockIdx.x + n * grid;
    return t < p.ntiles ? t : (int64_t)blockIdx.x;
  };
  uint32_t voff0[DPW];
  auto dma_off = [&](int j, int64_t last) -> uint32_t {
    const int d = wave * DPW + j;
    const bool sub1 = d * 1024 >= SUB1;
    const int ob = sub1 ? d * 1024 - SUB1 : d * 1024;
    const int gsub = (sub1 ? RB1 : RB0) / 16;
    const int gp = ob / 16 + lane;
    const int r = gp / gsub, jg = gp % gsub;
    const int64_t rr = r < last ? r : last;
    return (uint32_t)(rr * (sub1 ? p.lda1 : p.lda0) * 2 + 16 * (jg ^ (r & 15)));
  };
#pragma unroll
  for (int j = 0; j < DPW; ++j) voff0[j] = dma_off(j, TM);
  auto issue = [&](int64_t n) {
    const int64_t r0 = tile_of(n) * TM;
    const int64_t last = p.M - 1 - r0;
#pragma unroll
    for (int j = 0; j < DPW; ++j) {
      const int d = wave * DPW + j;
      const bool sub1 = d * 1024 >= SUB1;
      const char* base = reinterpret_cast<const char*>(sub1 ? p.a1 + r0 * p.lda1
                                                            : p.a0 + r0 * p.lda0);
      uint32_t la = lds0 + (uint32_t)((n % NBUF) * TB + d * 1024);
      asm volatile("" : "+s"(base), "+s"(la));
      dma16(base, last >= TM - 1 ? voff0[j] : dma_off(j, last), la);
    }
  };
#pragma unroll
  for (int n = 0; n < NBUF - 1; ++n) issue(n);

  const float inv_n = 1.0f / 256.f;
  const uint32_t dthr = sldm::dropout_threshold(p.drop_p);
  typedef __attribute__((address_space(3))) const s8v* lds_frag;

  f4v dv[RG][CT];              // previous tile: z - mean, MFMA layout
  int64_t tprev = 0;
  // ---- output work of the previous tile, in pieces ----
  float rs[RG];
  int64_t prow[RG];
  uint32_t rkey[RG];
  uint32_t wx[CT][2], wo[CT][2];
  auto out_prep = [&](int i) {
#pragma unroll
    for (int m = 0; m < RG; ++m) {
      const f4v* pr = reinterpret_cast<const f4v*>(red + (TM + 16 * m + i) * 8);
      const f4v a = pr[0], b = pr[1];
      const float tot = a[0] + a[1] + a[2] + a[3] + b[0] + b[1] + b[2] + b[3];
      rs[m] = 1.0f / sqrtf(tot * inv_n + p.eps);
      const int64_t row = tprev * TM + 16 * m + i;
      prow[m] = row < p.M ? row : p.M - 1;    // rows past M rewrite row M-1 (clamped loads)
      rkey[m] = sldm::dropout_row_key(p.seed, (uint64_t)(prow[m] + p.row_off));
    }
  };
  auto out_piece = [&](int m, int ct, int q) {
#if SLDM_WSLN_EXP == 4
    wx[ct][0] = wo[ct][0] = sldm::pack_bf16x2(dv[m][ct][0], dv[m][ct][1]);   // diagnostic
    wx[ct][1] = wo[ct][1] = sldm::pack_bf16x2(dv[m][ct][2], dv[m][ct][3]);
    return;
#endif
    const int c = cbase + 16 * ct + 4 * q;
    const f4v gg = *reinterpret_cast<const f4v*>(prm + 256 + c);
    const f4v be = *reinterpret_cast<const f4v*>(prm + 512 + c);
    bool keep[4];
    sldm::dropout_keep2(rkey[m], (uint32_t)c, dthr, keep[0], keep[1]);   // thr 0: all kept
    sldm::dropout_keep2(rkey[m], (uint32_t)c + 2, dthr, keep[2], keep[3]);
    float xh[4], o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      xh[r] = dv[m][ct][r] * rs[m];
      const float y = xh[r] * gg[r] + be[r];
      const float a = y > 0.f ? y : y * p.slope;
      o[r] = keep[r] ? a * p.drop_scale : 0.f;
    }
    wx[ct][0] = sldm::pack_bf16x2(xh[0], xh[1]);
    wx[ct][1] = sldm::pack_bf16x2(xh[2], xh[3]);
    wo[ct][0] = sldm::pack_bf16x2(o[0], o[1]);
    wo[ct][1] = sldm::pack_bf16x2(o[2], o[3]);
  };
  auto out_store = [&](int m, int q) {
    const int ccol = cbase + ((q & 1) ? 16 + 4 * (q - 1) : 4 * q);
    if constexpr (SAVE) {
      auto s0 = __builtin_amdgcn_permlane16_swap(wx[0][0], wx[1][0], false, false);
      auto s1 = __builtin_amdgcn_permlane16_swap(wx[0][1], wx[1][1], false, false);
      *reinterpret_cast<uint4*>(p.xhat + prow[m] * 256 + ccol) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
    auto s0 = __builtin_amdgcn_permlane16_swap(wo[0][0], wo[1][0], false, false);
    auto s1 = __builtin_amdgcn_permlane16_swap(wo[0][1], wo[1][1], false, false);
    *reinterpret_cast<uint4*>(p.out + prow[m] * 256 + ccol) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
  };
  auto out_rstd = [&]() {
    if constexpr (SAVE) {
      // one store per wave, every lane: lane l writes row l & 31 (lanes l and
      // l + 32 write the same value); rs[0] holds row i, rs[1] row 16 + i
      const int64_t row = tprev * TM + (lane & 31);
      p.rstd[row < p.M ? row : p.M - 1] = (lane & 16) ? rs[1] : rs[0];
    }
  };

  auto body = [&](int64_t n, auto has_prev_c) {
    constexpr bool HP = decltype(has_prev_c)::value;
    const int64_t tile = blockIdx.x + n * grid;
    int i, q;
    {
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      i = ln & 15;
      q = ln >> 4;
    }
    if (n < NBUF) wait_vm<VM_START>();
    else wait_vm<VM_STEADY>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(n + NBUF - 1);

    f4v acc[RG][CT];
#pragma unroll
    for (int m = 0; m < RG; ++m)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[m][ct] = f4v{0.f, 0.f, 0.f, 0.f};
    const uint32_t sl = lds0 + (uint32_t)((n % NBUF) * TB);
    uint32_t lb0[4], lb1[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t o = (uint32_t)(64 * (b ^ (i >> 2)) + 16 * ((q ^ i) & 3));
      lb0[b] = sl + (uint32_t)(i * RB0) + o;
      lb1[b] = sl + (uint32_t)(SUB1 + i * RB1) + o;
    }
    s8v bf[2][RG];
    auto read_b = [&](int s, s8v (&dst)[RG]) {
      const bool s1 = s >= K0STEPS;
      const int ls = s1 ? s - K0STEPS : s;
      const int rb = s1 ? RB1 : RB0;
      const uint32_t a = (s1 ? lb1 : lb0)[ls & 3] + (uint32_t)(256 * (ls >> 2));
#pragma unroll
      for (int m = 0; m < RG; ++m) dst[m] = *(lds_frag)(uintptr_t)(a + (uint32_t)(16 * m * rb));
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
      if constexpr (HP) {
        // the previous tile's output work, pinned between the k-steps
        if (s == 0) out_prep(i);
        if (s == 1 * SLOT8) out_piece(0, 0, q);
        if (s == 2 * SLOT8) out_piece(0, 1, q);
        if (s == 3 * SLOT8) out_store(0, q);
        if (s == 4 * SLOT8) out_piece(1, 0, q);
        if (s == 5 * SLOT8) out_piece(1, 1, q);
        if (s == 6 * SLOT8) out_store(1, q);
        if (s == 7 * SLOT8) out_rstd();
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // bias + row sums of this tile -> red[0]; barrier; deviations; squares -> red[1]
    float part[RG];
#pragma unroll
    for (int m = 0; m < RG; ++m) {
      part[m] = 0.f;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const f4v bb = *reinterpret_cast<const f4v*>(prm + cbase + 16 * ct + 4 * q);
        acc[m][ct] += bb;
#pragma unroll
        for (int r = 0; r < 4; ++r) part[m] += acc[m][ct][r];
      }
      const float v = sldm::row4_sum(part[m]);
#if SLDM_WSLN_EXP == 3
      part[m] = v;
#else
      if (q == 0) red[(16 * m + i) * 8 + wave] = v;
#endif
    }
#if SLDM_WSLN_EXP != 3
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
#pragma unroll
    for (int m = 0; m < RG; ++m) {
#if SLDM_WSLN_EXP == 3
      const float mean = part[m] * (8.f * inv_n);   // diagnostic: own partial only
#else
      const f4v* pr = reinterpret_cast<const f4v*>(red + (16 * m + i) * 8);
      const f4v a = pr[0], b = pr[1];
      const float mean = (a[0] + a[1] + a[2] + a[3] + b[0] + b[1] + b[2] + b[3]) * inv_n;
#endif
      float sq = 0.f;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[m][ct][r] - mean;
          dv[m][ct][r] = d;
          sq += d * d;
        }
      sq = sldm::row4_sum(sq);
      if (q == 0) red[(TM + 16 * m + i) * 8 + wave] = sq;
    }
    tprev = tile;
  };

  body(0, std::false_type{});
  int64_t n = 1;
  for (;; ++n) {
    if (blockIdx.x + n * grid >= p.ntiles) break;
    body(n, std::true_type{});
  }
  // the last tile's output work (its squared sums published by this barrier)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  {
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    const int i = ln & 15, q = ln >> 4;
    out_prep(i);
    out_piece(0, 0, q);
    out_piece(0, 1, q);
    out_store(0, q);
    out_piece(1, 0, q);
    out_piece(1, 1, q);
    out_store(1, q);
    out_rstd();
  }
  wait_vm<0>();
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

template <int KSTEPS, int K0STEPS, int NBUF>
int launch_ws_ln_pipe(WsLnArgs& p, bool save, hipStream_t stream) {
  constexpr int TM = 32;
  constexpr size_t lds = (size_t)NBUF * TM * KSTEPS * 64 + 3 * 256 * sizeof(float) +
                         (size_t)2 * TM * 8 * sizeof(float);
  static_assert(lds <= 160 * 1024, "LDS budget");
  p.ntiles = (p.M + TM - 1) / TM;
  const int64_t grid = std::min<int64_t>(p.ntiles, num_cus());
  auto kern = save ? ws_ln_pipe_kernel<KSTEPS, K0STEPS, NBUF, true>
                   : ws_ln_pipe_kernel<KSTEPS, K0STEPS, NBUF, false>;
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, kThreads, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("ws_ln_pipe_kernel");
  return SLDM_OK;
}

template <int KSTEPS, int K0STEPS, int NBUF, int TM, bool XCHG>
int launch_ws_ln(WsLnArgs& p, hipStream_t stream) {
  constexpr size_t lds = ws_ln_lds_bytes<KSTEPS, NBUF, TM, XCHG>();
  static_assert(lds <= 160 * 1024, "LDS budget");
  p.ntiles = (p.M + TM - 1) / TM;
  const int64_t grid = std::min<int64_t>(p.ntiles, num_cus());
  auto kern = ws_ln_kernel<KSTEPS, K0STEPS, NBUF, TM, XCHG>;
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, kThreads, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("ws_ln_kernel");
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
// The weight-stationary forward is opt-in (SLDM_WS_FWD=1): with each row's
// 256 columns spread over 8 waves its per-row epilogue work (statistics merge,
// dropout row key, addressing) is repeated by 32 lanes instead of 4, ~55 VALU
// instructions per output element against the stream kernel's ~15, and it
// measured 5.4-5.6 ms against 4.8 at C4.
// SLDM_WS_FWD=2 selects the statistics-exchange epilogue (no z round trip),
// 3 the same with the epilogue pipelined into the next tile's MFMAs.
int ws_fwd_mode() {
  const char* e = getenv("SLDM_WS_FWD");
  if (!ws_gemm_enabled() || !e) return 0;
  return e[0] == '1' ? 1 : (e[0] == '2' ? 2 : (e[0] == '3' ? 3 : 0));
}
bool ws_fwd_enabled() { return ws_fwd_mode() != 0; }

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
                     void* out, int64_t ldo, void* out2, int64_t ldo2, hipStream_t stream) {
  (void)k;
  WsArgs p{};
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

// Shape gate: bf16 (caller), 256 output columns, K = k0 + k1 of 256 or 512
// split on a 128-column boundary, contiguous [M][256] outputs, 16-B aligned
// rows and bases, 32-bit DMA offsets.
bool ws_dense_fwd_ok(int64_t k0, int64_t k1, int64_t nc, int64_t num_rows, const void* a0,
                     int64_t lda0, const void* a1, int64_t lda1, const void* w, const void* out,
                     const void* xhat) {
  const int64_t K = k0 + k1;
  if (nc != 256 || (K != 256 && K != 512) || k0 % 128 || k1 % 128) return false;
  if (num_rows >= (int64_t(1) << 30) || lda0 % 8 || lda0 > (1 << 20)) return false;
  if (k1 && (lda1 % 8 || lda1 > (1 << 20) || !aligned16(a1))) return false;
  return aligned16(a0) && aligned16(w) && aligned16(out) && (!xhat || aligned16(xhat));
}

int ws_dense_fwd(const void* a0, int64_t lda0, int64_t k0, const void* a1, int64_t lda1,
                 int64_t k1, const void* w, int64_t num_rows, const float* bias,
                 const float* gamma, const float* beta, float eps, float slope, float drop_p,
                 uint64_t seed, int64_t row_off, void* out, void* xhat, float* rstd,
                 hipStream_t stream) {
  WsLnArgs p{};
  p.a0 = (const uint16_t*)a0; p.lda0 = lda0;
  p.a1 = k1 ? (const uint16_t*)a1 : (const uint16_t*)a0; p.lda1 = k1 ? lda1 : lda0;
  p.w = (const uint16_t*)w;
  p.M = num_rows;
  p.out = (uint16_t*)out; p.xhat = (uint16_t*)xhat; p.rstd = rstd;
  p.bias = bias; p.gamma = gamma; p.beta = beta; p.eps = eps; p.slope = slope;
  p.drop_p = drop_p;
  p.drop_scale = drop_p >= 1.f ? 0.f : (drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f);
  p.seed = seed; p.row_off = row_off;
  const int64_t K = k0 + k1;
  if (ws_fwd_mode() == 3) {
    // the pipelined epilogue writes xhat and rstd together (or neither)
    const bool save = xhat != nullptr;
    if (save != (rstd != nullptr)) {
      sldm::set_error("ws_dense_fwd: xhat and rstd must be both given or both NULL");
      return SLDM_ERR_ARG;
    }
    if (K == 512) {
      if (k0 == 256) return launch_ws_ln_pipe<16, 8, 4>(p, save, stream);
      if (k0 == 128) return launch_ws_ln_pipe<16, 4, 4>(p, save, stream);
      if (k0 == 384) return launch_ws_ln_pipe<16, 12, 4>(p, save, stream);
      return launch_ws_ln_pipe<16, 16, 4>(p, save, stream);
    }
    if (k0 == 128) return launch_ws_ln_pipe<8, 4, 8>(p, save, stream);
    return launch_ws_ln_pipe<8, 8, 8>(p, save, stream);
  }
  if (ws_fwd_mode() == 1) {
    if (K == 512) {
      if (k0 == 256) return launch_ws_ln<16, 8, 3, 32, false>(p, stream);
      if (k0 == 128) return launch_ws_ln<16, 4, 3, 32, false>(p, stream);
      if (k0 == 384) return launch_ws_ln<16, 12, 3, 32, false>(p, stream);
      return launch_ws_ln<16, 16, 3, 32, false>(p, stream);
    }
    if (k0 == 128) return launch_ws_ln<8, 4, 4, 32, false>(p, stream);
    return launch_ws_ln<8, 8, 4, 32, false>(p, stream);
  }
  if (K == 512) {
    if (k0 == 256) return launch_ws_ln<16, 8, 4, 32, true>(p, stream);
    if (k0 == 128) return launch_ws_ln<16, 4, 4, 32, true>(p, stream);
    if (k0 == 384) return launch_ws_ln<16, 12, 4, 32, true>(p, stream);
    return launch_ws_ln<16, 16, 4, 32, true>(p, stream);
  }
  if (k0 == 128) return launch_ws_ln<8, 4, 8, 32, true>(p, stream);
  return launch_ws_ln<8, 8, 8, 32, true>(p, stream);
}

}  // namespace sldm
