// GRU over the vehicle trajectories: the model's
// torch.nn.GRU(dynamic_features_num -> gru_hidden_size, 1 layer, batch_first)
// (grusage.py:66-71, called at :160-161), forward and backward.
//
// torch's GRU (MIOpen) runs the T = 100 recurrence at ~1 % of the fp32 MFMA
// peak on the vehicle batch ([9600, 100, 6] -> 96, bench.py --config gru:
// 101 ms per fwd + bwd).  Here one workgroup owns a 16-row tile of sequences
// for the whole recurrence, one wave per 16 hidden units:
//
//  * the recurrent weights never leave registers: wave w holds the MFMA
//    B-fragments of W_hh rows {g*H + 16w + c} (gates r, z, n) for all k --
//    3 H/4 VGPRs -- and of W_ih likewise (3 KI);
//  * h_t lives in a double-buffered LDS image laid out as MFMA A-fragments
//    (one ds_read_b128 brings 4 k-steps), written by the wave that owns each
//    hidden tile, one barrier per step;
//  * per step and wave: KI + 3 H/4 ... x3 v_mfma_f32_16x16x4_f32 (exact fp32,
//    k-ordered fma chains; no reduced-precision path on gfx950), then the
//    gate math of its 16 x 16 outputs in registers: the r / z / n columns of
//    one hidden unit sit in the same lane of three accumulators.
//  PyTorch's cell (aten RNN.cpp gru_cell): r = s(gi_r + gh_r),
//  z = s(gi_z + gh_z), n = tanh(gi_n + r * gh_n), h' = (h - n) * z + n, with
//  gi = x W_ih^T + b_ih and gh = h W_hh^T + b_hh.
//
// The forward stores every h_t (the output) and, for the backward, the gate
// values r, z, n and gh_n in a lane-native workspace.  The backward runs the
// recurrence in reverse with the weight-gradient tiles dW_hh (3 H/4 regs),
// dW_ih, db as MFMA accumulators across all steps (the C-layout dGh is the A
// operand of dGh^T h_{t-1} with the 4 register rows as the k index) and
// W_hh's fragments for dh_{t-1} = dGh W_hh in LDS (beside the accumulators
// they would take the wave to 295 VGPRs); per-workgroup partials are summed
// by a reduce kernel in a fixed order (deterministic).
//
// Sizes: H = 16 NW (NW = 1..6 waves), I <= 16 (KI = ceil(I / 4) k-steps).
#include "common.hpp"

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef short s8b __attribute__((ext_vector_type(8)));   // 8 x bf16 (MFMA operand)

__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }

// LDS image of a [16 rows][K] operand as MFMA A-fragments: k-step q of lane l
// is element (row l & 15, k = 4q + (l >> 4)); four consecutive k-steps of a
// lane are one 16-B word: float index ((q >> 2) * 64 + l) * 4 + (q & 3).
__device__ __forceinline__ int aimg(int row, int k) {
  const int q = k >> 2, lane = row + 16 * (k & 3);
  return ((q >> 2) * 64 + lane) * 4 + (q & 3);
}


// The x operand of both forward kernels (A: row c, k = 4q + g4), staged in
// LDS TC steps at a time, double-buffered: chunk n + 2 is loaded into
// registers when chunk n + 1 is written to LDS, TC steps before any step reads
// it, so no step waits on a global load.  (Loaded one step ahead in registers,
// the compiler drained vmcnt -- the previous step's output and gate stores
// included -- at the top of every step: a store round trip per step.)  Both
// forward kernels are held to 168 VGPRs (3 waves per SIMD: two 6-wave
// workgroups per CU at H = 96) with the staging registers.
constexpr int x_chunk_steps(int nw, int ki) {
  return 4 * nw / ki >= 16 ? 16 : (4 * nw / ki >= 8 ? 8 : (4 * nw / ki >= 4 ? 4 : 2));
}
template <int NW, int KI>
struct XStage {
  static constexpr int TC = x_chunk_steps(NW, KI);
  static constexpr int CH = TC * KI * 64;                    // floats per chunk
  static constexpr int PT = (CH + 64 * NW - 1) / (64 * NW);  // per thread
  float r[PT];
  __device__ __forceinline__ void load(const float* __restrict__ x, int64_t ldxn, int64_t ldxt,
                                       int64_t N, int T, int I, int64_t r0, int t0) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int e = (int)threadIdx.x + i * 64 * NW;
      const int tt = e / (KI * 64), rem = e - tt * (KI * 64);
      const int k = 4 * (rem >> 6) + ((rem & 63) >> 4);
      const int t = t0 + tt;
      const int64_t xr = min(r0 + (rem & 15), N - 1);
      r[i] = (e < CH && k < I && t < T) ? x[xr * ldxn + (int64_t)t * ldxt + k] : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* buf) const {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int e = (int)threadIdx.x + i * 64 * NW;
      if (e < CH) buf[e] = r[i];
    }
  }
};

template <int NW, int KI>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(3))) void gru_fwd_kernel(
    const float* __restrict__ x, int64_t ldxn, int64_t ldxt, int64_t N, int T, int I,
    const float* __restrict__ w_ih, const float* __restrict__ w_hh,
    const float* __restrict__ b_ih, const float* __restrict__ b_hh,
    const float* __restrict__ h0, float* __restrict__ out, int64_t ldon, int64_t ldot,
    float* __restrict__ h_n, float* __restrict__ gates) {
  constexpr int H = 16 * NW;
  constexpr int KH = H / 4;                 // k-steps over the hidden dim
  __shared__ __attribute__((aligned(16))) float himg[2][KH * 64];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int c = lane & 15, g4 = lane >> 4;
  const int j = 16 * w + c;                 // this lane's hidden unit
  const int64_t r0 = (int64_t)blockIdx.x * 16;

  // weights (B-fragments: B[k = 4q + g4][col c] = W[g H + j][k])
  float whh[3][KH], wih[3][KI];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
#pragma unroll
    for (int q = 0; q < KH; ++q) whh[g][q] = w_hh[(int64_t)(g * H + j) * H + 4 * q + g4];
#pragma unroll
    for (int q = 0; q < KI; ++q) {
      const int k = 4 * q + g4;
      wih[g][q] = k < I ? w_ih[(int64_t)(g * H + j) * I + k] : 0.f;
    }
  }
  float bias[4];                            // r, z (ih + hh), n_ih, n_hh
  bias[0] = (b_ih ? b_ih[j] : 0.f) + (b_hh ? b_hh[j] : 0.f);
  bias[1] = (b_ih ? b_ih[H + j] : 0.f) + (b_hh ? b_hh[H + j] : 0.f);
  bias[2] = b_ih ? b_ih[2 * H + j] : 0.f;
  bias[3] = b_hh ? b_hh[2 * H + j] : 0.f;

  // own h (C-layout: rows 4 g4 + r, column j) and the initial LDS image
  float hp[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = r0 + 4 * g4 + r;
    hp[r] = (h0 && row < N) ? h0[row * H + j] : 0.f;
    himg[0][aimg(4 * g4 + r, j)] = hp[r];
  }
  // x operand (A: row c, k = 4q + g4) from the LDS chunks (XStage)
  using XS = XStage<NW, KI>;
  __shared__ __attribute__((aligned(16))) float xs[2][XS::CH];
  XS xst;
  xst.load(x, ldxn, ldxt, N, T, I, r0, 0);
  xst.store(xs[0]);
  xst.load(x, ldxn, ldxt, N, T, I, r0, XS::TC);
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const int tt = t % XS::TC;
    float xa[KI];
#pragma unroll
    for (int q = 0; q < KI; ++q) xa[q] = xs[(t / XS::TC) & 1][(tt * KI + q) * 64 + lane];
    const float* hi = himg[t & 1];
    f4v ar = {0.f, 0.f, 0.f, 0.f}, az = ar, an = ar, ahn = ar;
#pragma unroll
    for (int q = 0; q < KI; ++q) {
      ar = mfma4(xa[q], wih[0][q], ar);
      az = mfma4(xa[q], wih[1][q], az);
      an = mfma4(xa[q], wih[2][q], an);
    }
#pragma unroll
    for (int qq = 0; qq < KH / 4; ++qq) {
      const f4v a4 = *reinterpret_cast<const f4v*>(hi + (qq * 64 + lane) * 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = 4 * qq + u;
        ar = mfma4(a4[u], whh[0][q], ar);
        az = mfma4(a4[u], whh[1][q], az);
        ahn = mfma4(a4[u], whh[2][q], ahn);
      }
    }
    float* ho = himg[(t + 1) & 1];
    f4v gr, gz, gn, gh;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float rr = sigm(ar[r] + bias[0]);
      const float zz = sigm(az[r] + bias[1]);
      const float hn = ahn[r] + bias[3];
      const float nn = tanhf(an[r] + bias[2] + rr * hn);
      const float hv = (hp[r] - nn) * zz + nn;
      gr[r] = rr; gz[r] = zz; gn[r] = nn; gh[r] = hn;
      hp[r] = hv;
      ho[aimg(4 * g4 + r, j)] = hv;
      const int64_t row = r0 + 4 * g4 + r;
      if (row < N) out[row * ldon + (int64_t)t * ldot + j] = hv;
    }
    if (gates) {
      f4v* gp = reinterpret_cast<f4v*>(gates) +
                ((((int64_t)t * gridDim.x + blockIdx.x) * NW + w) * 4) * 64 + lane;
      gp[0] = gr; gp[64] = gz; gp[128] = gn; gp[192] = gh;
    }
    if (tt == XS::TC - 1 && t + 1 < T) {     // next chunk in, the one after loading
      xst.store(xs[(t / XS::TC + 1) & 1]);
      xst.load(x, ldxn, ldxt, N, T, I, r0, t + 1 + XS::TC);
    }
    __syncthreads();
  }
  if (h_n) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = r0 + 4 * g4 + r;
      if (row < N) h_n[row * H + j] = hp[r];
    }
  }
}

// Forward with the recurrent product h W_hh^T on bf16 MFMAs in split form
// ("bf16x3"): every fp32 operand x is carried as hi = bf16(x) plus
// lo = bf16(x - hi) (16 significant bits of 24), and a product as
// a_hi b_hi + a_hi b_lo + a_lo b_hi in fp32 accumulation -- the dropped
// a_lo b_lo and the split remainders are ~2^-16 relative, ~1e-5 on a gate's
// pre-activation (the GRU parity tests hold outputs and gradients to 1e-4
// against the fp32 oracle).  v_mfma_f32_16x16x32_bf16 does a 32-deep k-step in
// 16 cycles where the exact fp32 MFMA needs eight 16x16x4 steps of 32 cycles:
// the recurrence's MFMA time drops ~5x (3 k-steps x 3 products x 3 gates per
// step at H = 96, against 72 fp32 MFMAs).  The input product x W_ih^T (K <= 16)
// stays on the exact fp32 MFMA.  Layout: lane (c, g4) holds W_hh rows g H + j
// at k = 32 s + 8 g4 + e (e < 8) as the B operand, hi and lo (the same 72
// VGPRs as the fp32 kernel at H = 96); h_t sits in LDS as an fp32 image in the
// 16x16x32 A-operand layout and each reader splits its fragment.  Gate math,
// stores and the gates workspace are gru_fwd_kernel's.
using sldm::split_bf16x8;
// Gate nonlinearities of the split kernel on the hardware transcendentals
// (v_exp_f32, v_rcp_f32: ~1e-7 relative, far inside the 1e-4 bar): the
// libm expf / tanhf / division sequences were the longest part of a step.
__device__ __forceinline__ float fast_sigm(float v) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-v));
}
__device__ __forceinline__ float fast_tanh(float v) { return 2.0f * fast_sigm(2.0f * v) - 1.0f; }
__device__ __forceinline__ f4v mfma32(s8b a, s8b b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
typedef short s4b __attribute__((ext_vector_type(4)));   // 4 x bf16
__device__ __forceinline__ f4v mfma16(s4b a, s4b b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void split4(const float (&v)[4], s4b& hi, s4b& lo) {
  uint2 h, l;
  sldm::split_bf16x4(v, h, l);
  hi = __builtin_bit_cast(s4b, h);
  lo = __builtin_bit_cast(s4b, l);
}
// fp32 A-layout image of a [16 rows][KS*32] operand: element (row, k) of
// k-step s = k >> 5 sits in lane row + 16 ((k & 31) >> 3), slot k & 7.
__device__ __forceinline__ int aimg32(int row, int k) {
  return (((k >> 5) * 64 + row + 16 * ((k & 31) >> 3)) << 3) + (k & 7);
}

template <int NW, int KI>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(3))) void gru_fwd_x3_kernel(
    const float* __restrict__ x, int64_t ldxn, int64_t ldxt, int64_t N, int T, int I,
    const float* __restrict__ w_ih, const float* __restrict__ w_hh,
    const float* __restrict__ b_ih, const float* __restrict__ b_hh,
    const float* __restrict__ h0, float* __restrict__ out, int64_t ldon, int64_t ldot,
    float* __restrict__ h_n, float* __restrict__ gates) {
  constexpr int H = 16 * NW;
  constexpr int KS = (H + 31) / 32;         // 32-deep bf16 k-steps over the hidden dim
  constexpr int IMG = KS * 64 * 8;          // floats per image
  __shared__ __attribute__((aligned(16))) float himg[2][IMG];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int c = lane & 15, g4 = lane >> 4;
  const int j = 16 * w + c;
  const int64_t r0 = (int64_t)blockIdx.x * 16;

  s8b whi[3][KS], wlo[3][KS];
  float wih[3][KI];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 32 * s + 8 * g4 + e;
        v[e] = k < H ? w_hh[(int64_t)(g * H + j) * H + k] : 0.f;
      }
      split_bf16x8(v, whi[g][s], wlo[g][s]);
    }
#pragma unroll
    for (int q = 0; q < KI; ++q) {
      const int k = 4 * q + g4;
      wih[g][q] = k < I ? w_ih[(int64_t)(g * H + j) * I + k] : 0.f;
    }
  }
  float bias[4];
  bias[0] = (b_ih ? b_ih[j] : 0.f) + (b_hh ? b_hh[j] : 0.f);
  bias[1] = (b_ih ? b_ih[H + j] : 0.f) + (b_hh ? b_hh[H + j] : 0.f);
  bias[2] = b_ih ? b_ih[2 * H + j] : 0.f;
  bias[3] = b_hh ? b_hh[2 * H + j] : 0.f;

  if constexpr (H % 32 != 0) {              // zero k-padding of both images
    for (int e = threadIdx.x; e < 2 * IMG; e += 64 * NW) (&himg[0][0])[e] = 0.f;
    __syncthreads();
  }
  float hp[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = r0 + 4 * g4 + r;
    hp[r] = (h0 && row < N) ? h0[row * H + j] : 0.f;
    himg[0][aimg32(4 * g4 + r, j)] = hp[r];
  }
  using XS = XStage<NW, KI>;
  __shared__ __attribute__((aligned(16))) float xs[2][XS::CH];
  XS xst;
  xst.load(x, ldxn, ldxt, N, T, I, r0, 0);
  xst.store(xs[0]);
  xst.load(x, ldxn, ldxt, N, T, I, r0, XS::TC);
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const int tt = t % XS::TC;
    float xa[KI];
#pragma unroll
    for (int q = 0; q < KI; ++q) xa[q] = xs[(t / XS::TC) & 1][(tt * KI + q) * 64 + lane];
    const float* hi = himg[t & 1];
    f4v ar = {0.f, 0.f, 0.f, 0.f}, az = ar, an = ar, ahn = ar;
#pragma unroll
    for (int q = 0; q < KI; ++q) {
      ar = mfma4(xa[q], wih[0][q], ar);
      az = mfma4(xa[q], wih[1][q], az);
      an = mfma4(xa[q], wih[2][q], an);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const f4v* src = reinterpret_cast<const f4v*>(hi + ((s * 64 + lane) << 3));
      const f4v u0 = src[0], u1 = src[1];
      const float v[8] = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
      s8b ahi, alo;
      split_bf16x8(v, ahi, alo);
      ar = mfma32(alo, whi[0][s], ar);
      az = mfma32(alo, whi[1][s], az);
      ahn = mfma32(alo, whi[2][s], ahn);
      ar = mfma32(ahi, wlo[0][s], ar);
      az = mfma32(ahi, wlo[1][s], az);
      ahn = mfma32(ahi, wlo[2][s], ahn);
      ar = mfma32(ahi, whi[0][s], ar);
      az = mfma32(ahi, whi[1][s], az);
      ahn = mfma32(ahi, whi[2][s], ahn);
    }
    float* ho = himg[(t + 1) & 1];
    f4v gr, gz, gn, gh;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float rr = fast_sigm(ar[r] + bias[0]);
      const float zz = fast_sigm(az[r] + bias[1]);
      const float hn = ahn[r] + bias[3];
      const float nn = fast_tanh(an[r] + bias[2] + rr * hn);
      const float hv = (hp[r] - nn) * zz + nn;
      gr[r] = rr; gz[r] = zz; gn[r] = nn; gh[r] = hn;
      hp[r] = hv;
      ho[aimg32(4 * g4 + r, j)] = hv;
      const int64_t row = r0 + 4 * g4 + r;
      if (row < N) out[row * ldon + (int64_t)t * ldot + j] = hv;
    }
    if (gates) {
      f4v* gp = reinterpret_cast<f4v*>(gates) +
                ((((int64_t)t * gridDim.x + blockIdx.x) * NW + w) * 4) * 64 + lane;
      gp[0] = gr; gp[64] = gz; gp[128] = gn; gp[192] = gh;
    }
    if (tt == XS::TC - 1 && t + 1 < T) {     // next chunk in, the one after loading
      xst.store(xs[(t / XS::TC + 1) & 1]);
      xst.load(x, ldxn, ldxt, N, T, I, r0, t + 1 + XS::TC);
    }
    __syncthreads();
  }
  if (h_n) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = r0 + 4 * g4 + r;
      if (row < N) h_n[row * H + j] = hp[r];
    }
  }
}

// Backward.  Per step (t descending), wave w, lane (c, g4), rows 4 g4 + r:
//   dh   = carry + dout[t]           (carry = dh_n at t = T-1)
//   dn   = dh (1 - z),  dz = dh (h_{t-1} - n),  dh_{t-1} <- dh z
//   dan  = dn (1 - n^2), dr = dan gh_n, dar = dr r (1 - r), daz = dz z (1 - z)
//   dGi  = [dar, daz, dan],  dGh = [dar, daz, dan r]
//   dh_{t-1} += dGh W_hh                      (LDS image of dGh, W_hh frags)
//   dW_hh += dGh^T h_{t-1}, dW_ih += dGi^T x_t, db += column sums
template <int NW, int KI, bool X3, bool DGI>
__global__ __launch_bounds__(64 * NW) void gru_bwd_kernel(
    const float* __restrict__ x, int64_t ldxn, int64_t ldxt, int64_t N, int T, int I,
    const float* __restrict__ w_hh, const float* __restrict__ h0,
    const float* __restrict__ out, int64_t ldon, int64_t ldot, const float* __restrict__ gates,
    const float* __restrict__ dout, int64_t lddn, int64_t lddt, const float* __restrict__ dh_n,
    float* __restrict__ dh0, float* __restrict__ dgi, float* __restrict__ part) {
  constexpr int H = 16 * NW;
  constexpr int KG = 3 * H / 4;             // k-steps over the 3H gate columns
  // LDS (dynamic, gru_bwd_lds_bytes): dGh A-fragment image [2][KG*64],
  // h_{t-1} C-layout tiles [2][NW*256], and this workgroup's copy of the
  // dGh W_hh B-fragments [NW][KG/4][64][4] -- 3 H^2 floats (110.6 KB at
  // H = 96) that do not fit in registers beside the dW_hh accumulators.
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float (*gimg)[KG * 64] = reinterpret_cast<float (*)[KG * 64]>(lds);
  float (*pimg)[NW * 256] = reinterpret_cast<float (*)[NW * 256]>(lds + 2 * KG * 64);
  float* wimg = lds + 2 * KG * 64 + 2 * NW * 256;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int c = lane & 15, g4 = lane >> 4;
  const int j = 16 * w + c;
  const int64_t r0 = (int64_t)blockIdx.x * 16;

  // B-fragments of dGh W_hh: B[k = gate column 4q + g4][col j] = W_hh[4q + g4][j]
  // (X3: 32-deep k-steps, lane (c, g4) k = 32 s + 8 g4 + e, as bf16 hi | lo)
  constexpr int KS3 = 3 * H / 32;           // X3 k-steps over the 3H gate columns
  static_assert(!X3 || (3 * H) % 32 == 0, "split form: 3H a multiple of 32");
  float* wmine = wimg + (int64_t)w * KG * 64;
  if constexpr (X3) {
    uint4* wq = reinterpret_cast<uint4*>(wmine);
    for (int s3 = 0; s3 < KS3; ++s3) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = w_hh[(int64_t)(32 * s3 + 8 * g4 + e) * H + j];
      s8b hi, lo;
      split_bf16x8(v, hi, lo);
      wq[(s3 * 64 + lane) * 2] = __builtin_bit_cast(uint4, hi);
      wq[(s3 * 64 + lane) * 2 + 1] = __builtin_bit_cast(uint4, lo);
    }
  } else {
#pragma unroll 4
    for (int q = 0; q < KG; ++q)
      wmine[((q >> 2) * 64 + lane) * 4 + (q & 3)] = w_hh[(int64_t)(4 * q + g4) * H + j];
  }

  f4v dwh[3][NW], dwi[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    dwi[g] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NW; ++kt) dwh[g][kt] = f4v{0.f, 0.f, 0.f, 0.f};
  }
  float db[4] = {0.f, 0.f, 0.f, 0.f};       // r, z, n_ih, n_hh column sums

  bool live[4];
  float dh[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = r0 + 4 * g4 + r;
    live[r] = row < N;
    dh[r] = (dh_n && live[r]) ? dh_n[row * H + j] : 0.f;
  }
  // Step operands (saved gates, h_{t-1}, dout[t], x[t]) are loaded one step
  // ahead, every load unconditional (clamped rows, sources and strides picked
  // by scalar selects, values masked after the load) and every store of the loop unconditional
  // (dgi has padded rows, DGI a template parameter): with a fixed op count per
  // step the compiler's vmcnt waits release exactly the step they feed.  (With
  // conditional loads and stores its bookkeeping fell back to waiting for the
  // loads it had just issued: a global round trip per step.)
  struct StepIn {
    f4v gr, gz, gn, gh;
    float hp[4], go[4], xb[4];
  };
  const int ci = c < I ? c : I - 1;
  // source bases and strides chosen once (scalar selects), so the per-step
  // addresses are plain arithmetic: h_{t-1} from out (t > 0) or h0 (t = 0;
  // out again as a dummy when h0 is absent), dout likewise
  const float* const h0p = h0 ? h0 : out;
  const int64_t h0s = h0 ? H : ldon;
  const float* const dp = dout ? dout : out;
  const int64_t dsn = dout ? lddn : ldon, dst = dout ? lddt : 0;
  auto load_step = [&](int t, StepIn& in) {
    const bool tp = t > 0;
    const float* const hb = tp ? out : h0p;   // (t = 0 without h0: a dummy row of out)
    const int64_t hsn = tp ? ldon : h0s, hst = tp ? (int64_t)(t - 1) * ldot : 0;
    const f4v* gp = reinterpret_cast<const f4v*>(gates) +
                    ((((int64_t)t * gridDim.x + blockIdx.x) * NW + w) * 4) * 64 + lane;
    in.gr = gp[0]; in.gz = gp[64]; in.gn = gp[128]; in.gh = gp[192];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = min(r0 + 4 * g4 + r, N - 1);
      // raw values: the masks are applied where the step consumes them (a
      // select here lets the compiler skip -- i.e. branch around -- the load)
      in.hp[r] = hb[row * hsn + hst + j];
      in.go[r] = dp[row * dsn + (int64_t)t * dst + j];
      // x as the B operand of dW_ih: B[k <-> row 4 g4 + r][col i = c]
      in.xb[r] = x[row * ldxn + (int64_t)t * ldxt + ci];
    }
  };
  StepIn nxt;
  load_step(T - 1, nxt);
  for (int t = T - 1; t >= 0; --t) {
    const int b = t & 1;
    const StepIn cur = nxt;
    load_step(t > 0 ? t - 1 : 0, nxt);   // at step 0: a harmless re-load
    const f4v gr = cur.gr, gz = cur.gz, gn = cur.gn, gh = cur.gh;
    float hp[4], xb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      hp[r] = (t > 0 || h0) ? cur.hp[r] : 0.f;
      xb[r] = c < I ? cur.xb[r] : 0.f;
      dh[r] += (dout && live[r]) ? cur.go[r] : 0.f;
    }
    f4v dar, daz, dan, dghn;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = live[r] ? dh[r] : 0.f;
      const float dn = d * (1.f - gz[r]);
      const float dz = d * (hp[r] - gn[r]);
      const float an = dn * (1.f - gn[r] * gn[r]);
      const float drr = an * gh[r];
      dar[r] = drr * gr[r] * (1.f - gr[r]);
      daz[r] = dz * gz[r] * (1.f - gz[r]);
      dan[r] = an;
      dghn[r] = an * gr[r];
      dh[r] = d * gz[r];                    // direct path; + dGh W_hh below
      db[0] += dar[r];
      db[1] += daz[r];
      db[2] += dan[r];
      db[3] += dghn[r];
      // dGh image (A-fragments over the 3H gate columns) and h_{t-1} tile
      if constexpr (X3) {
        gimg[b][aimg32(4 * g4 + r, j)] = dar[r];
        gimg[b][aimg32(4 * g4 + r, H + j)] = daz[r];
        gimg[b][aimg32(4 * g4 + r, 2 * H + j)] = dghn[r];
      } else {
        gimg[b][aimg(4 * g4 + r, j)] = dar[r];
        gimg[b][aimg(4 * g4 + r, H + j)] = daz[r];
        gimg[b][aimg(4 * g4 + r, 2 * H + j)] = dghn[r];
      }
    }
    *reinterpret_cast<f4v*>(&pimg[b][(w * 64 + lane) * 4]) = f4v{hp[0], hp[1], hp[2], hp[3]};
    if constexpr (DGI) {                    // dx needs dGi: [rows, T, 3H] in (row, t) order
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // rows past N land in the workspace's padding rows (unconditional)
        const int64_t row = r0 + 4 * g4 + r;
        float* o = dgi + (row * T + t) * (int64_t)(3 * H);
        o[j] = dar[r];
        o[H + j] = daz[r];
        o[2 * H + j] = dan[r];
      }
    }
    __syncthreads();

    // dh_{t-1} += dGh W_hh (rows 4 g4 + r, column j)
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    const float* gi = gimg[b];
    if constexpr (X3) {
      const uint4* wq = reinterpret_cast<const uint4*>(wmine);
#pragma unroll
      for (int s3 = 0; s3 < KS3; ++s3) {
        const f4v* src = reinterpret_cast<const f4v*>(gi + ((s3 * 64 + lane) << 3));
        const f4v u0 = src[0], u1 = src[1];
        const float v[8] = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
        s8b ahi, alo;
        split_bf16x8(v, ahi, alo);
        const s8b bhi = __builtin_bit_cast(s8b, wq[(s3 * 64 + lane) * 2]);
        const s8b blo = __builtin_bit_cast(s8b, wq[(s3 * 64 + lane) * 2 + 1]);
        acc = mfma32(alo, bhi, acc);
        acc = mfma32(ahi, blo, acc);
        acc = mfma32(ahi, bhi, acc);
      }
    } else {
#pragma unroll
      for (int qq = 0; qq < KG / 4; ++qq) {
        const f4v a4 = *reinterpret_cast<const f4v*>(gi + (qq * 64 + lane) * 4);
        const f4v b4 = *reinterpret_cast<const f4v*>(wmine + (qq * 64 + lane) * 4);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = mfma4(a4[u], b4[u], acc);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) dh[r] += acc[r];

    // dW_hh[g H + 16 w + c'][16 kt + c''] += sum_rows dGh h_{t-1}: A = this
    // lane's dGh registers (k-step r <-> row 4 g4 + r), B = h_{t-1} tile kt
    if constexpr (X3) {
      // The 16 rows of a step are exactly the K = 16 of one
      // v_mfma_f32_16x16x16_bf16 (lane (c, g4) supplies k = 4 g4 + r, the
      // same rows the four fp32 16x16x4 steps take): split form, three bf16
      // MFMAs per tile instead of four fp32 ones -- the weight-gradient
      // accumulation was the longest MFMA chain of a step (6 x 3 tiles).
      const float va[3][4] = {{dar[0], dar[1], dar[2], dar[3]},
                              {daz[0], daz[1], daz[2], daz[3]},
                              {dghn[0], dghn[1], dghn[2], dghn[3]}};
      s4b ahi[3], alo[3];
#pragma unroll
      for (int g = 0; g < 3; ++g) split4(va[g], ahi[g], alo[g]);
#pragma unroll
      for (int kt = 0; kt < NW; ++kt) {
        const f4v hb = *reinterpret_cast<const f4v*>(&pimg[b][(kt * 64 + lane) * 4]);
        const float vb[4] = {hb[0], hb[1], hb[2], hb[3]};
        s4b bhi, blo;
        split4(vb, bhi, blo);
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          dwh[g][kt] = mfma16(alo[g], bhi, dwh[g][kt]);
          dwh[g][kt] = mfma16(ahi[g], blo, dwh[g][kt]);
          dwh[g][kt] = mfma16(ahi[g], bhi, dwh[g][kt]);
        }
      }
      const float vx[4] = {xb[0], xb[1], xb[2], xb[3]};
      const float vn[4] = {dan[0], dan[1], dan[2], dan[3]};
      s4b xhi, xlo, nhi, nlo;
      split4(vx, xhi, xlo);
      split4(vn, nhi, nlo);
      const s4b* aih[3] = {&ahi[0], &ahi[1], &nhi};
      const s4b* ail[3] = {&alo[0], &alo[1], &nlo};
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        dwi[g] = mfma16(*ail[g], xhi, dwi[g]);
        dwi[g] = mfma16(*aih[g], xlo, dwi[g]);
        dwi[g] = mfma16(*aih[g], xhi, dwi[g]);
      }
    } else {
#pragma unroll
      for (int kt = 0; kt < NW; ++kt) {
        const f4v hb = *reinterpret_cast<const f4v*>(&pimg[b][(kt * 64 + lane) * 4]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dwh[0][kt] = mfma4(dar[r], hb[r], dwh[0][kt]);
          dwh[1][kt] = mfma4(daz[r], hb[r], dwh[1][kt]);
          dwh[2][kt] = mfma4(dghn[r], hb[r], dwh[2][kt]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dwi[0] = mfma4(dar[r], xb[r], dwi[0]);
        dwi[1] = mfma4(daz[r], xb[r], dwi[1]);
        dwi[2] = mfma4(dan[r], xb[r], dwi[2]);
      }
    }
  }
  if (dh0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = r0 + 4 * g4 + r;
      if (live[r]) dh0[row * H + j] = dh[r];
    }
  }
  // per-workgroup partials: [3H][H] dW_hh | [3H][16] dW_ih | [4][H] db
  // (accumulator D[row c'][col c''] = lane c'' of register 4 g4 + i)
  float* p = part + (int64_t)blockIdx.x * (3 * H * H + 3 * H * 16 + 4 * H);
#pragma unroll
  for (int g = 0; g < 3; ++g) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int crow = g * H + 16 * w + 4 * g4 + i;
#pragma unroll
      for (int kt = 0; kt < NW; ++kt) p[crow * H + 16 * kt + c] = dwh[g][kt][i];
      p[3 * H * H + crow * 16 + c] = dwi[g][i];
    }
  }
  // column sums: reduce the four row groups (g4) of each column
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float v = db[k];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (g4 == 0) p[3 * H * H + 3 * H * 16 + k * H + j] = v;
  }
}

// Sum the per-workgroup partials in workgroup order (deterministic) into
// dW_hh [3H][H], dW_ih [3H][I], db_ih [3H], db_hh [3H].
__global__ __launch_bounds__(256) void gru_reduce_kernel(const float* __restrict__ part,
                                                         int64_t nparts, int H, int I,
                                                         float* __restrict__ dw_ih,
                                                         float* __restrict__ dw_hh,
                                                         float* __restrict__ db_ih,
                                                         float* __restrict__ db_hh) {
  const int64_t stride = 3 * H * H + 3 * H * 16 + 4 * H;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= stride) return;
  // eight interleaved partial chains (loads in flight), then combined in a
  // fixed order: deterministic
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int64_t p = 0;
  for (; p + 8 <= nparts; p += 8)
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += part[(p + u) * stride + e];
  for (; p < nparts; ++p) a[0] += part[p * stride + e];
  const float s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  if (e < 3 * H * H) {
    dw_hh[e] = s;
    return;
  }
  int64_t f = e - 3 * H * H;
  if (f < 3 * H * 16) {
    const int64_t crow = f / 16, i = f % 16;
    if (i < I) dw_ih[crow * I + i] = s;
    return;
  }
  f -= 3 * H * 16;
  const int k = (int)(f / H), jj = (int)(f % H);
  // k: 0 = r (ih and hh), 1 = z (ih and hh), 2 = n_ih, 3 = n_hh
  if (k < 2) {
    if (db_ih) db_ih[k * H + jj] = s;
    if (db_hh) db_hh[k * H + jj] = s;
  } else if (k == 2) {
    if (db_ih) db_ih[2 * H + jj] = s;
  } else if (db_hh) {
    db_hh[2 * H + jj] = s;
  }
}

// dx[n, t, i] = sum_c dGi[n, t, c] W_ih[c, i]  (only when x needs a gradient)
__global__ __launch_bounds__(256) void gru_dx_kernel(const float* __restrict__ dgi,
                                                     const float* __restrict__ w_ih, int64_t rows,
                                                     int H, int I, float* __restrict__ dx,
                                                     int64_t T, int64_t lddxn, int64_t lddxt) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * I) return;
  const int64_t rt = e / I;
  const int i = (int)(e % I);
  const float* g = dgi + rt * 3 * H;
  float s = 0.f;
  for (int k = 0; k < 3 * H; ++k) s = fmaf(g[k], w_ih[(int64_t)k * I + i], s);
  const int64_t n = rt / T, t = rt % T;
  dx[n * lddxn + t * lddxt + i] = s;
}

// The split-bf16 recurrent product (gru_fwd_x3_kernel) is the default;
// SLDM_GRU_BF16X3=0 selects the exact fp32 MFMA kernel (read per call).
bool gru_bf16x3_enabled() {
  const char* e = getenv("SLDM_GRU_BF16X3");
  return !(e && e[0] == '0');
}

template <int NW>
int launch_fwd(int ki, dim3 grid, hipStream_t st, const float* x, int64_t ldxn, int64_t ldxt,
               int64_t N, int T, int I, const float* w_ih, const float* w_hh, const float* b_ih,
               const float* b_hh, const float* h0, float* out, int64_t ldon, int64_t ldot,
               float* h_n, float* gates) {
#define SLDM_GRU_F(KI)                                                                         \
  if (gru_bf16x3_enabled())                                                                    \
    gru_fwd_x3_kernel<NW, KI><<<grid, 64 * NW, 0, st>>>(x, ldxn, ldxt, N, T, I, w_ih, w_hh,    \
                                                        b_ih, b_hh, h0, out, ldon, ldot, h_n, \
                                                        gates);                               \
  else                                                                                         \
    gru_fwd_kernel<NW, KI><<<grid, 64 * NW, 0, st>>>(x, ldxn, ldxt, N, T, I, w_ih, w_hh, b_ih, \
                                                     b_hh, h0, out, ldon, ldot, h_n, gates)
  switch (ki) {
    case 1: SLDM_GRU_F(1); break;
    case 2: SLDM_GRU_F(2); break;
    case 3: SLDM_GRU_F(3); break;
    default: SLDM_GRU_F(4); break;
  }
#undef SLDM_GRU_F
  SLDM_LAUNCH_CHECK("gru_fwd_kernel");
  return SLDM_OK;
}

template <int NW>
int launch_bwd(dim3 grid, hipStream_t st, const float* x, int64_t ldxn, int64_t ldxt, int64_t N,
               int T, int I, const float* w_hh, const float* h0, const float* out, int64_t ldon,
               int64_t ldot, const float* gates, const float* dout, int64_t lddn, int64_t lddt,
               const float* dh_n, float* dh0, float* dgi, float* part) {
  constexpr int H = 16 * NW;
  constexpr size_t lds = sizeof(float) * (2 * (3 * H / 4) * 64 + 2 * NW * 256 + 3 * H * H);
  static_assert(lds <= 160 * 1024, "GRU backward LDS budget");
  // the split form needs the 3H gate columns in whole 32-deep k-steps
  // (H = 32, 64, 96); other sizes run the fp32 MFMA recurrence
  auto kern = dgi ? gru_bwd_kernel<NW, 1, false, true> : gru_bwd_kernel<NW, 1, false, false>;
  if constexpr ((3 * H) % 32 == 0) {
    if (gru_bf16x3_enabled())
      kern = dgi ? gru_bwd_kernel<NW, 1, true, true> : gru_bwd_kernel<NW, 1, true, false>;
  }
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  kern<<<grid, 64 * NW, lds, st>>>(x, ldxn, ldxt, N, T, I, w_hh, h0, out, ldon, ldot, gates,
                                   dout, lddn, lddt, dh_n, dh0, dgi, part);
  SLDM_LAUNCH_CHECK("gru_bwd_kernel");
  return SLDM_OK;
}

bool gru_shape_ok(int64_t N, int64_t T, int64_t I, int64_t H) {
  return N > 0 && T > 0 && I >= 1 && I <= 16 && H >= 16 && H <= 96 && H % 16 == 0 &&
         N < ((int64_t)1 << 31) && T < ((int64_t)1 << 24);
}

}  // namespace

extern "C" size_t sldm_gru_workspace_bytes(int64_t N, int64_t T, int64_t H) {
  if (N <= 0 || T <= 0 || H <= 0) return 16;
  const int64_t tiles = (N + 15) / 16;
  return (size_t)(T * tiles * (H / 16) * 4 * 64 * 4) * sizeof(float);
}

extern "C" int sldm_gru_fwd(const float* x, int64_t ldx_n, int64_t ldx_t, int64_t N, int64_t T,
                            int64_t I, int64_t H, const float* w_ih, const float* w_hh,
                            const float* b_ih, const float* b_hh, const float* h0, float* out,
                            int64_t ldo_n, int64_t ldo_t, float* h_n, float* gates,
                            void* stream_) {
  SLDM_REQUIRE(gru_shape_ok(N, T, I, H),
               "sldm_gru_fwd: unsupported shape N=%lld T=%lld I=%lld H=%lld (1 <= I <= 16, "
               "H in 16..96 a multiple of 16)", (long long)N, (long long)T, (long long)I,
               (long long)H);
  SLDM_REQUIRE(x && w_ih && w_hh && out, "sldm_gru_fwd: NULL argument");
  hipStream_t st = sldm::as_stream(stream_);
  const dim3 grid((unsigned)((N + 15) / 16));
  const int ki = (int)((I + 3) / 4);
  const int t = (int)T, i = (int)I;
  switch (H / 16) {
    case 1: return launch_fwd<1>(ki, grid, st, x, ldx_n, ldx_t, N, t, i, w_ih, w_hh, b_ih, b_hh, h0, out, ldo_n, ldo_t, h_n, gates);
    case 2: return launch_fwd<2>(ki, grid, st, x, ldx_n, ldx_t, N, t, i, w_ih, w_hh, b_ih, b_hh, h0, out, ldo_n, ldo_t, h_n, gates);
    case 3: return launch_fwd<3>(ki, grid, st, x, ldx_n, ldx_t, N, t, i, w_ih, w_hh, b_ih, b_hh, h0, out, ldo_n, ldo_t, h_n, gates);
    case 4: return launch_fwd<4>(ki, grid, st, x, ldx_n, ldx_t, N, t, i, w_ih, w_hh, b_ih, b_hh, h0, out, ldo_n, ldo_t, h_n, gates);
    case 5: return launch_fwd<5>(ki, grid, st, x, ldx_n, ldx_t, N, t, i, w_ih, w_hh, b_ih, b_hh, h0, out, ldo_n, ldo_t, h_n, gates);
    default: return launch_fwd<6>(ki, grid, st, x, ldx_n, ldx_t, N, t, i, w_ih, w_hh, b_ih, b_hh, h0, out, ldo_n, ldo_t, h_n, gates);
  }
}

extern "C" size_t sldm_gru_bwd_workspace_bytes(int64_t N, int64_t T, int64_t I, int64_t H,
                                               int need_dx) {
  if (N <= 0 || T <= 0 || H <= 0) return 16;
  const int64_t tiles = (N + 15) / 16;
  size_t b = (size_t)tiles * (3 * H * H + 3 * H * 16 + 4 * H) * sizeof(float);
  // dGi rows padded to whole 16-row tiles (the backward stores them unconditionally)
  if (need_dx) b += (size_t)tiles * 16 * T * 3 * H * sizeof(float);
  return b;
}

extern "C" int sldm_gru_bwd(const float* x, int64_t ldx_n, int64_t ldx_t, int64_t N, int64_t T,
                            int64_t I, int64_t H, const float* w_ih, const float* w_hh,
                            const float* h0, const float* out, int64_t ldo_n, int64_t ldo_t,
                            const float* gates, const float* dout, int64_t ldd_n, int64_t ldd_t,
                            const float* dh_n, float* dx, int64_t lddx_n, int64_t lddx_t,
                            float* dh0, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh,
                            void* workspace, size_t workspace_bytes, void* stream_) {
  SLDM_REQUIRE(gru_shape_ok(N, T, I, H), "sldm_gru_bwd: unsupported shape");
  SLDM_REQUIRE(x && w_ih && w_hh && out && gates && dw_ih && dw_hh && workspace,
               "sldm_gru_bwd: NULL argument");
  SLDM_REQUIRE(workspace_bytes >= sldm_gru_bwd_workspace_bytes(N, T, I, H, dx != nullptr),
               "sldm_gru_bwd: workspace too small");
  hipStream_t st = sldm::as_stream(stream_);
  const int64_t tiles = (N + 15) / 16;
  const dim3 grid((unsigned)tiles);
  float* part = reinterpret_cast<float*>(workspace);
  float* dgi = dx ? part + tiles * (3 * H * H + 3 * H * 16 + 4 * H) : nullptr;
  const int t = (int)T, i = (int)I;
  int rc;
  switch (H / 16) {
    case 1: rc = launch_bwd<1>(grid, st, x, ldx_n, ldx_t, N, t, i, w_hh, h0, out, ldo_n, ldo_t, gates, dout, ldd_n, ldd_t, dh_n, dh0, dgi, part); break;
    case 2: rc = launch_bwd<2>(grid, st, x, ldx_n, ldx_t, N, t, i, w_hh, h0, out, ldo_n, ldo_t, gates, dout, ldd_n, ldd_t, dh_n, dh0, dgi, part); break;
    case 3: rc = launch_bwd<3>(grid, st, x, ldx_n, ldx_t, N, t, i, w_hh, h0, out, ldo_n, ldo_t, gates, dout, ldd_n, ldd_t, dh_n, dh0, dgi, part); break;
    case 4: rc = launch_bwd<4>(grid, st, x, ldx_n, ldx_t, N, t, i, w_hh, h0, out, ldo_n, ldo_t, gates, dout, ldd_n, ldd_t, dh_n, dh0, dgi, part); break;
    case 5: rc = launch_bwd<5>(grid, st, x, ldx_n, ldx_t, N, t, i, w_hh, h0, out, ldo_n, ldo_t, gates, dout, ldd_n, ldd_t, dh_n, dh0, dgi, part); break;
    default: rc = launch_bwd<6>(grid, st, x, ldx_n, ldx_t, N, t, i, w_hh, h0, out, ldo_n, ldo_t, gates, dout, ldd_n, ldd_t, dh_n, dh0, dgi, part); break;
  }
  if (rc != SLDM_OK) return rc;
  const int64_t stride = 3 * H * H + 3 * H * 16 + 4 * H;
  gru_reduce_kernel<<<(unsigned)((stride + 255) / 256), 256, 0, st>>>(
      part, tiles, (int)H, i, dw_ih, dw_hh, db_ih, db_hh);
  SLDM_LAUNCH_CHECK("gru_reduce_kernel");
  if (dx) {
    const int64_t rows = N * T;
    gru_dx_kernel<<<(unsigned)((rows * I + 255) / 256), 256, 0, st>>>(dgi, w_ih, rows, (int)H,
                                                                       i, dx, T, lddx_n, lddx_t);
    SLDM_LAUNCH_CHECK("gru_dx_kernel");
  }
  return SLDM_OK;
}
