// Persistent "register-A" bf16 MFMA kernels for the dense part of a SageBlock
// layer at F_out = 256 (forward) and the 1/deg-prescaled dX GEMM (backward).
//
// Same contractions and epilogues as gemm_big.hip, restructured for a GEMM
// whose K (256 | 512) is too short to amortise a per-tile prologue and
// epilogue, i.e. one that must stream HBM like a copy kernel:
//
//  * one 512-thread workgroup per CU loops over 256-row (128-row for the
//    two-column-group dX shape) tiles; the k-step sequence runs on across tile
//    boundaries, so the next tile's activation loads are in flight while the
//    current tile's epilogue computes and stores;
//  * activations never touch LDS: each wave owns 32 full rows and loads its
//    MFMA B-operand fragments (16 B per lane, 64 B per row per k-step) straight
//    from HBM into a 4-deep register ring; only the weights stream through
//    LDS, by LDS-DMA, in a 4-stage ring of 32-deep k-slices (same swizzled
//    image as gemm_big.hip) behind one counted `s_waitcnt vmcnt` + raw
//    s_barrier per k-step;
//  * a wave holds complete 256-column rows, so LayerNorm statistics reduce
//    in-wave (two xor shuffles), with no LDS exchange and no block barrier in
//    the epilogue; the LN outputs leave as 16-byte stores, each lane's two
//    4-column fragments of adjacent tiles paired by v_permlane16_swap (8
//    columns contiguous per lane, 16 rows x 64 B per store instruction;
//    row-per-lane 8-byte stores are store-issue-bound, MI355X_MICROARCH.md
//    "epilogue store tail").  Same-box A/B at C4 (tools/ab_run1.sh): 4.74 ms
//    against 4.79 ms through a per-wave LDS staging tile (SLDM_LN_STAGE=1,
//    whole-row stores, 67 KB of LDS and an LDS round trip per output).
//
// vmcnt bookkeeping: per k-step every wave issues WIPW weight DMAs then 2
// activation loads, so the slice consumed at step s is followed by exactly
// 2*WIPW+6 younger vector-memory ops (VM_BASE).  The first NSTW-1 steps of a
// tile other than the block's first additionally have the previous tile's
// epilogue stores (>= S_EPI of them, all rows of a non-final tile are real)
// younger than their slice, hence the looser VM_FIRST there.  Extra younger
// ops only make a count stricter, never unsafe.
#include "common.hpp"

namespace {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vptr;

// LN forward launch shape: waves per workgroup (8: one 512-thread workgroup
// per CU; 4: two 256-thread workgroups per CU, whose k-step barriers are
// independent, so one workgroup's epilogue VALU can overlap the other's loads
// -- measured slower, 5.38 vs 4.90 ms at C4: with 128-row tiles every CU
// streams the 256 KB weight matrix from L2 twice as often) and whether its outputs leave through the LDS staging tile (1) or as
// permlane16-paired 16-B stores (0; no staging LDS, required for 4 waves).
#ifndef SLDM_LN_NW
#define SLDM_LN_NW 8
#endif
#ifndef SLDM_LN_STAGE
#define SLDM_LN_STAGE 0
#endif
constexpr int RW = 32;            // rows per wave
constexpr int NTT = 16;           // 16-column MFMA tiles per wave (256 columns)
constexpr int NSTW = 4;           // weight ring stages
// Activation register ring depth (k-steps of A in flight per wave).  Any
// DA >= NSTW keeps the steady-state count VM_BASE: A(s) is issued DA steps
// ahead, before W(s) (NSTW-1 steps ahead), so the ops younger than W(s) are
// the same 2 W + 3 A groups (header comment).
#ifndef SLDM_STREAM_DA
#define SLDM_STREAM_DA 4
#endif

// Diagnostic builds only (tools/ab_build.sh): 1 = the LN kernel storing z
// without LayerNorm / activation / dropout (results wrong).
#ifndef SLDM_STREAM_EXP
#define SLDM_STREAM_EXP 0
#endif
constexpr int SROW = 512 + 16;    // LN staging row stride in bytes (conflict-free b64 writes)

enum { ST_LN = 0, ST_ROWSCALE = 1 };

struct StreamArgs {
  const uint16_t* a0; int64_t lda0; int k0;   // A columns [0, k0)
  const uint16_t* a1; int64_t lda1;           // A columns [k0, K)
  const uint16_t* b; int64_t ldb;             // B [Nc][K] (weights)
  int64_t M; int Nc; int64_t ntiles;
  uint16_t* out; int64_t ldo;
  uint16_t* xhat; float* rstd;
  const float* bias; const float* gamma; const float* beta;
  float eps, slope, drop_p, drop_scale; sldm::Seed seed; int64_t row_off;
  const int32_t* rowptr; int scale_cols;
  uint16_t* out2; int64_t ldo2;               // ROWSCALE: optional home of columns >= scale_cols
};

__device__ __forceinline__ int swz(int r16) { return (r16 >> 2) & 2; }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Same wait, ordering the two register-ring fragments it releases: their
// loads are hidden from the compiler (below), so this asm is what makes
// them "defined" for the MFMAs that follow.
template <int N>
__device__ __forceinline__ void wait_vm(s8v& a, s8v& b) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
// Every vector-memory op of the steady state is opaque asm in saddr form
// (uniform 64-bit SGPR base + 32-bit per-lane byte offset): activation
// fragments, degree words and the weight-slice LDS-DMA.  With compiler-visible
// LDS-DMA and VGPR loads both pending in vmcnt the waitcnt pass treats the
// counter as out of order and drains it (vmcnt(0)) before each use; here the
// kernel counts every op itself (header comment) and the compiler sees none.
__device__ __forceinline__ s8v gload16(const void* sbase, uint32_t voff) {
  s8v r;
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r) : "v"(voff), "s"(sbase) : "memory");
  return r;
}
__device__ __forceinline__ int gload4(const void* sbase, uint32_t voff) {
  int r;
  asm volatile("global_load_dword %0, %1, %2" : "=v"(r) : "v"(voff), "s"(sbase) : "memory");
  return r;
}
// 64 lanes x 16 B from sbase + voff[lane] to LDS [m0 .. m0 + 1 KB), lane-linear.
__device__ __forceinline__ void dma16(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
}

template <int KSTEPS, int WN, int MODE, int NW = 8, bool STAGE = true>
constexpr size_t stream_lds_bytes() {
  return (size_t)NSTW * 256 * WN * 64 +
         (MODE == ST_LN ? 3 * 256 * sizeof(float) + (STAGE ? NW * 16 * SROW : 0) : 0);
}

template <int KSTEPS, int WN, int MODE, bool SPLIT, bool HASDEG, int NW = 8, bool STAGE = true,
          int DA = SLDM_STREAM_DA>
__global__ __launch_bounds__(NW * 64, 2) void gemm_stream_kernel(StreamArgs p) {
  constexpr int NT_ = NW * 64;               // threads per workgroup
  constexpr int WR = NW / WN;                // row groups of 32 per tile
  constexpr int BM = WR * RW;                // rows per tile
  constexpr int WCOLS = 256 * WN;            // weight rows staged per k-step
  constexpr int WSTAGE = WCOLS * 64;         // bytes per weight slice
  constexpr int WIPW = WCOLS / (NW * 16);    // weight DMA instructions per wave per k-step
  static_assert(WCOLS % (NW * 16) == 0, "weight DMA rounds");
  constexpr int VM_BASE = 2 * WIPW + 6;
  // lower bound on epilogue vm ops per tile: LN 2 x 16 row stores (with
  // xhat, see loose_ok), ROWSCALE 2 x NTT/2 paired 16-B stores
  constexpr int S_EPI = MODE == ST_LN ? 32 : NTT;
  constexpr int VM_FIRST = VM_BASE + S_EPI > 63 ? 63 : VM_BASE + S_EPI;
  static_assert(KSTEPS % NSTW == 0 && KSTEPS % DA == 0 && KSTEPS >= NSTW && DA >= NSTW,
                "ring shape");
  static_assert(MODE == ST_ROWSCALE || WN == 1, "LN needs the whole row in one wave");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wring = smem;
  float* prm = reinterpret_cast<float*>(smem + NSTW * WSTAGE);   // bias | gamma | beta
  char* stage_base = smem + NSTW * WSTAGE + 3 * 256 * sizeof(float);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WN, wr = wave / WN;
  int q = lane >> 4, r16 = lane & 15;   // re-laundered per tile (see loop head)

  int64_t tile = blockIdx.x;
  if (tile >= p.ntiles) return;

  if constexpr (MODE == ST_LN) {
    for (int i = tid; i < 256; i += NT_) {
      prm[i] = p.bias ? p.bias[i] : 0.f;
      prm[256 + i] = p.gamma[i];
      prm[512 + i] = p.beta[i];
    }
    __syncthreads();   // before any DMA is in flight
  }

  // ---- weight slice DMA (same lane-linear swizzled image as gemm_big.hip) ---
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ swz(drow);
  // This lane's byte offset in W for DMA j = 0; DMA j adds the uniform
  // 128 W rows * ldb (on the scalar base): one VGPR for all WIPW DMAs.
  const uint32_t woff = (uint32_t)(((wave * 16 + drow) * (uint32_t)p.ldb + 8 * dchunk) * 2);
  const uint32_t wstride = (uint32_t)(NW * 16) * (uint32_t)p.ldb * 2u;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_vptr)smem;   // LDS byte address
  auto issue_w = [&](int slot, int ks) {
    // bases laundered before the constant parts are added: otherwise every
    // (step, DMA) address is hoisted into an SGPR of its own and spilled
    const char* wb = reinterpret_cast<const char*>(p.b);
    uint32_t la = lds0;
    asm volatile("" : "+s"(wb), "+s"(la));
    wb += ks * 64;
    la += slot * WSTAGE + wave * 16 * 64;
#pragma unroll
    for (int j = 0; j < WIPW; ++j) dma16(wb + j * wstride, woff, la + j * NW * 16 * 64);
  };
  // ---- activation fragments: lane (r16, q) <- row r16 (+16m), k 8q..8q+7 ----
  // Row pointers are formed once per tile; every k-step offset below is a
  // compile-time immediate (A = [a0 | a1] splits at K/2 when SPLIT).
  // A tile base (uniform, per half) + 32-bit per-lane row offsets; the k
  // offset goes on the scalar base.  Rows past M are clamped to M-1.
  struct TileA { const char* base0; const char* base1; uint32_t off[2]; };
  auto rows_of = [&](int64_t tl, TileA& ta) {
    const int64_t r0 = tl * BM;
    ta.base0 = reinterpret_cast<const char*>(p.a0 + r0 * p.lda0);
    ta.base1 = SPLIT ? reinterpret_cast<const char*>(p.a1 + r0 * p.lda1) : ta.base0;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int64_t row = min(r0 + wr * RW + 16 * m + r16, p.M - 1);
      ta.off[m] = (uint32_t)(((row - r0) * p.lda0 + 8 * q) * 2);
    }
  };
  auto load_a = [&](const TileA& ta, int ks, s8v (&dst)[2]) {
    const int kk = ks * 32;
    const bool h = SPLIT && kk >= KSTEPS * 16;
    const char* b = (h ? ta.base1 : ta.base0) + 2 * (h ? kk - KSTEPS * 16 : kk);
#pragma unroll
    for (int m = 0; m < 2; ++m) dst[m] = gload16(b, ta.off[m]);
  };

  s8v ar[DA][2];
  f4v acc[2][NTT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < NTT; ++t) acc[m][t] = f4v{0.f, 0.f, 0.f, 0.f};

  {
    TileA p0;
    rows_of(tile, p0);
    // Same issue order as the steady state (A(s+1) right after W(s)), so the
    // first tile's steps use the same counts: A(0), then W(s), A(s+1); the
    // remaining ring slots (DA > NSTW) after them -- younger ops only make
    // the first steps' counts stricter.
    load_a(p0, 0, ar[0]);
#pragma unroll
    for (int s = 0; s < NSTW - 1; ++s) {
      issue_w(s, s);
      load_a(p0, s + 1, ar[s + 1]);
    }
#pragma unroll
    for (int s = NSTW; s < DA; ++s) load_a(p0, s, ar[s]);
  }

  // The loose first-steps count is valid only when the previous epilogue
  // issued >= S_EPI vm ops: always in ROWSCALE (NTT = 16 stores), in LN only
  // when xhat is written too (2 x 16 stores).
  const bool loose_ok = MODE == ST_ROWSCALE || p.xhat != nullptr;
  bool first = true;
  for (;;) {
    // Lane id re-derived per tile by a volatile v_mbcnt pair (no inputs, so
    // nothing lane-derived is live across the loop and nothing per-lane is
    // tile-invariant for LICM to hoist into a table and spill).
    {
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      q = ln >> 4;
      r16 = ln & 15;
    }
    const int roff = 16 * (q ^ swz(r16));
    const int64_t nraw = tile + gridDim.x;
    const bool has_next = nraw < p.ntiles;
    const int64_t next = has_next ? nraw : tile;
    // row pointers live only while loads use them (recomputed, not carried
    // across the epilogue)
    TileA pcur, pnext;
    rows_of(tile, pcur);

    int dg[2][2] = {{0, 1}, {0, 1}};
    if constexpr (HASDEG) {
      // degree prefetch for this tile's rows (consumed by the epilogue)
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int64_t row = min(tile * BM + wr * RW + 16 * m + r16, p.M - 1);
        dg[m][0] = gload4(p.rowptr, (uint32_t)(row * 4));
        dg[m][1] = gload4(p.rowptr, (uint32_t)(row * 4 + 4));
      }
    }

#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      // A(ks) is older than W(ks), so this count releases both; the degree
      // loads (older than every W of this tile) are complete from ks = NSTW-1 on.
      if (ks < NSTW - 1 && !first && loose_ok) wait_vm<VM_FIRST>(ar[ks % DA][0], ar[ks % DA][1]);
      else wait_vm<VM_BASE>(ar[ks % DA][0], ar[ks % DA][1]);
      if constexpr (HASDEG) {
        if (ks == KSTEPS - 1)
          asm volatile("" : "+v"(dg[0][0]), "+v"(dg[0][1]), "+v"(dg[1][0]), "+v"(dg[1][1]));
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue_w((ks + NSTW - 1) % NSTW, (ks + NSTW - 1) % KSTEPS);
      const char* cur = wring + (ks % NSTW) * WSTAGE + (wc * 256 + r16) * 64 + roff;
#pragma unroll
      for (int t = 0; t < NTT; ++t) {
        const s8v wf = *reinterpret_cast<const s8v*>(cur + 16 * t * 64);
#pragma unroll
        for (int m = 0; m < 2; ++m)
          acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, ar[ks % DA][m], acc[m][t],
                                                              0, 0, 0);
      }
      if (ks == KSTEPS - DA) rows_of(next, pnext);
      if (ks + DA < KSTEPS) load_a(pcur, ks + DA, ar[ks % DA]);
      else load_a(pnext, ks + DA - KSTEPS, ar[ks % DA]);
      // Pin the step's schedule: two W fragments ahead, then one ds_read per
      // MFMA pair, so only ~3 fragments are live beside the 128 accumulators.
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int t = 0; t < NTT - 2; ++t) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }

    // ---- epilogue: acc[m][t][r] = C[row 16m + r16][col wc*256 + 16t + 4q + r]
    if constexpr (MODE == ST_LN) {
      char* stg = stage_base + wave * 16 * SROW;
      (void)stg;
      const float inv_n = 1.0f / 256.f;
      const uint32_t dthr = sldm::dropout_threshold(p.drop_p);
      const int cq = 4 * q;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        // Rows past M (final tile only) computed row M-1's values from its
        // clamped loads; clamping the row index everywhere (dropout key
        // included) makes their stores identical rewrites of row M-1.
        const int64_t row0 = tile * BM + wr * RW + 16 * m;   // first row of this 16-row slab
        const int64_t row = min(row0 + r16, p.M - 1);
#if SLDM_STREAM_EXP == 1
        const float rs = 1.f;   // diagnostic build: no LayerNorm / activation / dropout
        const uint32_t rkey = 0;
        (void)rkey;
#else
        // acc <- acc + bias; mean; acc <- (acc - mean); var; acc <- acc * rstd = xhat
        float s = 0.f;
#pragma unroll
        for (int t = 0; t < NTT; ++t) {
          const f4v bb = *reinterpret_cast<const f4v*>(prm + 16 * t + 4 * q);
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
#pragma unroll
        for (int t = 0; t < NTT; ++t) acc[m][t] *= rs;
        const uint32_t rkey = sldm::dropout_row_key(sldm::effective_seed(p.seed), (uint64_t)(row + p.row_off));
#endif
        if (p.rstd && q == 0) p.rstd[row] = rs;

        if constexpr (STAGE) {
          // two staging rounds through the wave's 16 x 512 B tile: xhat, then out
#pragma unroll
          for (int pass = 0; pass < 2; ++pass) {
            uint16_t* dst = pass == 0 ? p.xhat : p.out;
            if (pass == 0 && !dst) continue;
#pragma unroll
            for (int t = 0; t < NTT; ++t) {
              const int c = 16 * t + cq;
              float v[4];
              if (pass == 0 || SLDM_STREAM_EXP == 1) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[m][t][r];
              } else {
                const f4v gg = *reinterpret_cast<const f4v*>(prm + 256 + c);
                const f4v be = *reinterpret_cast<const f4v*>(prm + 512 + c);
                bool keep[4] = {true, true, true, true};
                if (p.drop_p > 0.f) {
                  sldm::dropout_keep2(rkey, (uint32_t)c, dthr, keep[0], keep[1]);
                  sldm::dropout_keep2(rkey, (uint32_t)c + 2, dthr, keep[2], keep[3]);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const float y = acc[m][t][r] * gg[r] + be[r];
                  const float a = fmaxf(y, y * p.slope);   // slope in [0, 1] (host-checked)
                  v[r] = keep[r] ? a * p.drop_scale : 0.f;
                }
              }
              sldm::Vec<uint16_t, 4>::store(reinterpret_cast<uint16_t*>(stg + r16 * SROW + 2 * c),
                                            v);
              if (t & 1) __builtin_amdgcn_sched_barrier(0);   // bound hoisted prm reads
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const int rr = 2 * i + (q >> 1);          // lane >> 5 (laundered ids)
              const int cb = ((q & 1) * 16 + r16) * 16; // (lane & 31) * 16
              const uint4 val = *reinterpret_cast<const uint4*>(stg + rr * SROW + cb);
              const int64_t drow_ = min(row0 + rr, p.M - 1);
              *reinterpret_cast<uint4*>(reinterpret_cast<char*>(dst + drow_ * p.ldo) + cb) = val;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
        } else {
          // permlane16-paired 16-B stores straight from the accumulators (the
          // ROWSCALE epilogue's pattern below): a store instruction covers 16
          // rows x 64 B, no staging LDS and no LDS round trip
#pragma unroll
          for (int pass = 0; pass < 2; ++pass) {
            uint16_t* dst = pass == 0 ? p.xhat : p.out;
            if (pass == 0 && !dst) continue;
#pragma unroll
            for (int t = 0; t < NTT; t += 2) {
              uint32_t w[2][2];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const int c = 16 * (t + h) + cq;
                float v[4];
                if (pass == 0 || SLDM_STREAM_EXP == 1) {
#pragma unroll
                  for (int r = 0; r < 4; ++r) v[r] = acc[m][t + h][r];
                } else {
                  const f4v gg = *reinterpret_cast<const f4v*>(prm + 256 + c);
                  const f4v be = *reinterpret_cast<const f4v*>(prm + 512 + c);
                  bool keep[4] = {true, true, true, true};
                  if (p.drop_p > 0.f) {
                    sldm::dropout_keep2(rkey, (uint32_t)c, dthr, keep[0], keep[1]);
                    sldm::dropout_keep2(rkey, (uint32_t)c + 2, dthr, keep[2], keep[3]);
                  }
#pragma unroll
                  for (int r = 0; r < 4; ++r) {
                    const float y = acc[m][t + h][r] * gg[r] + be[r];
                    const float a = fmaxf(y, y * p.slope);   // slope in [0, 1] (host-checked)
                    v[r] = keep[r] ? a * p.drop_scale : 0.f;
                  }
                }
                w[h][0] = sldm::pack_bf16x2(v[0], v[1]);
                w[h][1] = sldm::pack_bf16x2(v[2], v[3]);
              }
              auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
              auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
              const uint4 o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
              const int cc = 16 * t + ((q & 1) ? 16 + 4 * (q - 1) : 4 * q);
              *reinterpret_cast<uint4*>(dst + row * p.ldo + cc) = o;
              __builtin_amdgcn_sched_barrier(0);   // bound hoisted prm reads
            }
          }
        }
      }
    } else {
      // Split output (host-checked: scale_cols a multiple of 256, ldo2 == ldo):
      // a wave's 256 columns all go to one buffer, so only its uniform base
      // moves and no second per-lane row offset is live.
      uint16_t* obase = p.out;
      if (p.out2 && wc * 256 >= p.scale_cols) obase = p.out2 - p.scale_cols;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        // clamped like the loads: rows past M rewrite row M-1's own values
        const int64_t row = min(tile * BM + wr * RW + 16 * m + r16, p.M - 1);
        const int deg = dg[m][1] - dg[m][0];
        // 1/deg once per row (the 64-row kernels divide; the difference is
        // <= 1 fp32 ulp before the bf16 rounding)
        const float inv = HASDEG ? 1.0f / (float)(deg > 0 ? deg : 1) : 1.f;
        // Tiles t, t+1 leave together as one 16-B store per lane: a lane
        // holds 4 columns of each; v_permlane16_swap trades the odd row of
        // the first operand with the even row of the second, so lanes of even
        // q end with 8 contiguous columns of tile t (theirs + partner q+1's),
        // lanes of odd q with 8 of tile t+1 (partner q-1's + theirs) -- half
        // the store instructions of 8-B stores (store-issue-bound epilogue,
        // MI355X_MICROARCH.md "epilogue store tail").
#pragma unroll
        for (int t = 0; t < NTT; t += 2) {
          uint32_t w[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            // scale_cols (= F_in) is a multiple of 16: one uniform test per tile
            const bool scaled = wc * 256 + 16 * (t + h) < p.scale_cols;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = scaled ? acc[m][t + h][r] * inv : acc[m][t + h][r];
            w[h][0] = sldm::pack_bf16x2(v[0], v[1]);
            w[h][1] = sldm::pack_bf16x2(v[2], v[3]);
          }
          uint4 o;
          {
            auto s0 = __builtin_amdgcn_permlane16_swap(w[0][0], w[1][0], false, false);
            auto s1 = __builtin_amdgcn_permlane16_swap(w[0][1], w[1][1], false, false);
            o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
          }
          const int c = wc * 256 + 16 * t + ((q & 1) ? 16 + 4 * (q - 1) : 4 * q);
          *reinterpret_cast<uint4*>(obase + row * p.ldo + c) = o;
        }
      }
    }

    if (!has_next) break;
    tile = next;
    first = false;
#pragma unroll
    for (int i = 0; i < 2 * NTT; ++i) acc[i / NTT][i % NTT] = f4v{0.f, 0.f, 0.f, 0.f};
  }
  wait_vm<0>();   // retire the tail's dummy loads and weight DMAs
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

template <int KSTEPS, int WN, int MODE, bool SPLIT, bool HASDEG = false>
int launch_stream(StreamArgs& p, hipStream_t stream) {
  constexpr int NW = MODE == ST_LN ? SLDM_LN_NW : 8;
  constexpr bool STAGE = MODE == ST_LN ? SLDM_LN_STAGE != 0 : true;
  constexpr int BM = (NW / WN) * RW;
  constexpr size_t lds = stream_lds_bytes<KSTEPS, WN, MODE, NW, STAGE>();
  constexpr int per_cu = 8 / NW;       // workgroups per CU (two waves per SIMD)
  static_assert(lds * per_cu <= 160 * 1024, "LDS budget");
  p.ntiles = (p.M + BM - 1) / BM;
  const int64_t grid = std::min<int64_t>(p.ntiles, (int64_t)per_cu * num_cus());
  auto kern = gemm_stream_kernel<KSTEPS, WN, MODE, SPLIT, HASDEG, NW, STAGE>;
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<(unsigned)grid, NW * 64, lds, stream>>>(p);
  SLDM_LAUNCH_CHECK("gemm_stream_kernel");
  return SLDM_OK;
}

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

}  // namespace

namespace sldm {

bool stream_gemm_enabled() {
  static const bool on = [] {
    const char* e = getenv("SLDM_STREAM_GEMM");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Shape gate: bf16, K of 256 or 512 (k0 a multiple of the 32-deep k-step),
// 16-byte aligned rows and bases.
static bool stream_common_ok(int64_t k0, int64_t K, const void* a0, int64_t lda0, const void* a1,
                             int64_t lda1, const void* b, int64_t ldb) {
  if ((K != 256 && K != 512) || (k0 != K && 2 * k0 != K)) return false;
  if (k0 != K && lda1 != lda0) return false;   // one row offset serves both halves
  if (lda0 % 8 || (K > k0 && lda1 % 8) || ldb % 8) return false;
  return aligned16(a0) && (K == k0 || aligned16(a1)) && aligned16(b);
}

// The LN epilogue evaluates LeakyReLU as max(y, slope * y): equal to
// (y > 0 ? y : slope * y), signed zeros and NaN included, for slope in [0, 1]
// (ReLU and every leaky slope in use); other slopes take the tile kernels.
bool stream_dense_fwd_ok(int64_t k0, int64_t K, int64_t nc, const void* a0, int64_t lda0,
                         const void* a1, int64_t lda1, const void* w, const void* out,
                         const void* xhat, float slope) {
  return nc == 256 && slope >= 0.f && slope <= 1.f &&
         stream_common_ok(k0, K, a0, lda0, a1, lda1, w, K) && aligned16(out) &&
         (!xhat || aligned16(xhat));
}

bool stream_rowscale_ok(int64_t k, int64_t nc, const void* a, int64_t lda, const void* b,
                        int64_t ldb, const void* out, int64_t ldo, int64_t scale_cols) {
  return (nc == 256 || nc == 512) && ldo % 8 == 0 && scale_cols % 16 == 0 &&
         stream_common_ok(k, k, a, lda, a, lda, b, ldb) && aligned16(out);
}

int stream_dense_fwd(const void* a0, int64_t lda0, int64_t k0, const void* a1, int64_t lda1,
                     int64_t k1, const void* w, int64_t num_rows, const float* bias,
                     const float* gamma, const float* beta, float eps, float slope, float drop_p,
                     uint64_t seed, int64_t row_off, void* out, void* xhat, float* rstd,
                     hipStream_t stream) {
  StreamArgs p{};
  p.a0 = (const uint16_t*)a0; p.lda0 = lda0; p.k0 = (int)k0;
  p.a1 = k1 ? (const uint16_t*)a1 : (const uint16_t*)a0; p.lda1 = k1 ? lda1 : lda0;
  const int K = (int)(k0 + k1);
  p.b = (const uint16_t*)w; p.ldb = K;
  p.M = num_rows; p.Nc = 256;
  p.out = (uint16_t*)out; p.ldo = 256; p.xhat = (uint16_t*)xhat; p.rstd = rstd;
  p.bias = bias; p.gamma = gamma; p.beta = beta; p.eps = eps; p.slope = slope;
  p.drop_p = drop_p;
  p.drop_scale = drop_p >= 1.f ? 0.f : (drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f);
  p.seed = seed; p.row_off = row_off;
  if (k1 == 0)
    return K == 512 ? launch_stream<16, 1, ST_LN, false>(p, stream)
                    : launch_stream<8, 1, ST_LN, false>(p, stream);
  return K == 512 ? launch_stream<16, 1, ST_LN, true>(p, stream)
                  : launch_stream<8, 1, ST_LN, true>(p, stream);
}

int stream_gemm_rowscale(const void* a, int64_t lda, int64_t k, const void* b, int64_t ldb,
                         int64_t num_rows, int64_t nc, const int32_t* rowptr, int64_t scale_cols,
                         void* out, int64_t ldo, void* out2, int64_t ldo2, hipStream_t stream) {
  StreamArgs p{};
  p.a0 = (const uint16_t*)a; p.lda0 = lda; p.k0 = (int)k;
  p.a1 = (const uint16_t*)a; p.lda1 = lda;
  p.b = (const uint16_t*)b; p.ldb = ldb;
  p.M = num_rows; p.Nc = (int)nc;
  p.out = (uint16_t*)out; p.ldo = ldo;
  p.out2 = (uint16_t*)out2; p.ldo2 = ldo2;
  p.rowptr = rowptr; p.scale_cols = (int)scale_cols;
  auto go = [&](auto hasdeg) -> int {
    constexpr bool HD = decltype(hasdeg)::value;
    if (nc == 512)
      return k == 512 ? launch_stream<16, 2, ST_ROWSCALE, false, HD>(p, stream)
                      : launch_stream<8, 2, ST_ROWSCALE, false, HD>(p, stream);
    return k == 512 ? launch_stream<16, 1, ST_ROWSCALE, false, HD>(p, stream)
                    : launch_stream<8, 1, ST_ROWSCALE, false, HD>(p, stream);
  };
  return rowptr ? go(std::true_type{}) : go(std::false_type{});
}

}  // namespace sldm
