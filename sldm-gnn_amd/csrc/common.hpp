// Shared helpers for the gfx950 kernels of libsldm_sage.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "sldm_sage.h"

namespace sldm {

// Thread-local last-error message (sldm_last_error()).
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();
// Zero `words` 32-bit words at `ptr` with a kernel on `stream` (not a memset
// node: every launch of the library may be recorded into a HIP graph).
int zero_words(void* ptr, size_t words, void* stream);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;  // CDNA wavefront

// ------------------------------------------------------------------ bf16 --
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// Round-to-nearest-even; a plain cast lowers to v_cvt_pk_bf16_f32 on gfx950
// and keeps NaN a NaN.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
// Two values, one v_cvt_pk_bf16_f32 (same rounding): written as a 2-vector
// conversion because two scalar casts joined by shift / or lower to two
// converts (each against a zero half) plus the shift and an SDWA or.
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// The value a float becomes once stored as T (bf16: rounded; fp32: itself).
template <typename T> __device__ __forceinline__ float stored_value(float v);
template <> __device__ __forceinline__ float stored_value<float>(float v) { return v; }
template <> __device__ __forceinline__ float stored_value<uint16_t>(float v) {
  return bf16_to_f32(f32_to_bf16(v));
}

// ------------------------------------------- vector load/store of V elems --
// Loads V consecutive elements of T (float or uint16 bf16) into fp32 regs.
template <typename T, int V> struct Vec;

template <> struct Vec<float, 4> {
  __device__ static void load(const float* p, float* r) {
    float4 v = *reinterpret_cast<const float4*>(p);
    r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
  }
  __device__ static void store(float* p, const float* r) {
    *reinterpret_cast<float4*>(p) = make_float4(r[0], r[1], r[2], r[3]);
  }
};
template <> struct Vec<float, 2> {
  __device__ static void load(const float* p, float* r) {
    float2 v = *reinterpret_cast<const float2*>(p);
    r[0] = v.x; r[1] = v.y;
  }
  __device__ static void store(float* p, const float* r) {
    *reinterpret_cast<float2*>(p) = make_float2(r[0], r[1]);
  }
};
template <> struct Vec<float, 1> {
  __device__ static void load(const float* p, float* r) { r[0] = *p; }
  __device__ static void store(float* p, const float* r) { *p = r[0]; }
};
template <> struct Vec<uint16_t, 8> {
  __device__ static void load(const uint16_t* p, float* r) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    r[0] = bf16_lo(v.x); r[1] = bf16_hi(v.x); r[2] = bf16_lo(v.y); r[3] = bf16_hi(v.y);
    r[4] = bf16_lo(v.z); r[5] = bf16_hi(v.z); r[6] = bf16_lo(v.w); r[7] = bf16_hi(v.w);
  }
  __device__ static void store(uint16_t* p, const float* r) {
    *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]),
                                              pack_bf16x2(r[4], r[5]), pack_bf16x2(r[6], r[7]));
  }
};
template <> struct Vec<uint16_t, 4> {
  __device__ static void load(const uint16_t* p, float* r) {
    uint2 v = *reinterpret_cast<const uint2*>(p);
    r[0] = bf16_lo(v.x); r[1] = bf16_hi(v.x); r[2] = bf16_lo(v.y); r[3] = bf16_hi(v.y);
  }
  __device__ static void store(uint16_t* p, const float* r) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]));
  }
};
template <> struct Vec<uint16_t, 2> {
  __device__ static void load(const uint16_t* p, float* r) {
    uint32_t v = *reinterpret_cast<const uint32_t*>(p);
    r[0] = bf16_lo(v); r[1] = bf16_hi(v);
  }
  __device__ static void store(uint16_t* p, const float* r) {
    *reinterpret_cast<uint32_t*>(p) = pack_bf16x2(r[0], r[1]);
  }
};
template <> struct Vec<uint16_t, 1> {
  __device__ static void load(const uint16_t* p, float* r) { r[0] = bf16_to_f32(*p); }
  __device__ static void store(uint16_t* p, const float* r) { *p = f32_to_bf16(r[0]); }
};

// 16-B vector load / store with an optional non-temporal hint, for the gathers
// over tables far larger than the 256 MB Infinity Cache.  Same-box A/B of the
// C4 bench (nt_gather below): output stores non-temporal gain 2-3 % on the
// uniform graph and 2 % on the locality variant; adding non-temporal source
// loads matches that on the uniform graph but costs 10 % on the locality
// variant (its rows do reuse the cache), so the default is stores only.
// Other widths fall back to Vec.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <typename T, int V, bool NT>
__device__ __forceinline__ void load_vec(const T* p, float* r) {
  if constexpr (NT && sizeof(T) * V == 16) {
    const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { r[2 * i] = bf16_lo(w[i]); r[2 * i + 1] = bf16_hi(w[i]); }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = __uint_as_float(w[i]);
    }
  } else {
    Vec<T, V>::load(p, r);
  }
}
template <typename T, int V, bool NT>
__device__ __forceinline__ void store_vec(T* p, const float* r) {
  if constexpr (NT && sizeof(T) * V == 16) {
    u32x4 w;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = pack_bf16x2(r[2 * i], r[2 * i + 1]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = __float_as_uint(r[i]);
    }
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
  } else {
    Vec<T, V>::store(p, r);
  }
}
// Gathers switch to non-temporal access when the gathered table (estimated as
// rows x leading dimension: the graphs here are square) reaches this size.
// Mode bits: 1 = output stores, 2 = source-row loads.  SLDM_GATHER_NT in the
// environment forces a mode: 0 none, s stores only, 1 both (read per call).
constexpr int64_t kNtTableBytes = (int64_t)1 << 30;
// Per-row streamed operands of the gathers (the addend row, the LN backward's
// xhat row): loaded non-temporal too in the non-temporal (GiB-table) mode.
// Same-box A/B at C4 (kbench): fused layer boundary 12.10 -> 11.52 ms,
// transpose gather + addend 10.49 -> 10.34 ms, forward gather unchanged.
#ifndef SLDM_STREAM_OPERANDS_NT
#define SLDM_STREAM_OPERANDS_NT 1
#endif
constexpr bool kStreamOperandsNt = SLDM_STREAM_OPERANDS_NT != 0;
inline int nt_gather(int64_t table_bytes) {
  const char* e = getenv("SLDM_GATHER_NT");
  if (e && e[0] == '0') return 0;
  if (e && e[0] == 's') return 1;
  if (e && e[0] == '1') return 3;
  return table_bytes >= kNtTableBytes ? 1 : 0;
}

// Widest element count V (16 B max per lane) such that feat, the leading
// dimensions and the base pointers keep every V-vector naturally aligned.
inline int pick_vec(int elem_bytes, int64_t feat, std::initializer_list<int64_t> lds,
                    std::initializer_list<const void*> ptrs) {
  int v = 16 / elem_bytes;
  for (; v > 1; v >>= 1) {
    bool ok = (feat % v) == 0;
    for (int64_t ld : lds) ok = ok && (ld % v) == 0;
    for (const void* p : ptrs)
      ok = ok && (p == nullptr || (reinterpret_cast<uintptr_t>(p) % (size_t)(v * elem_bytes)) == 0);
    if (ok) break;
  }
  return v;
}

// Lanes that share one row: next power of two >= feat/V, capped at one wave.
inline int lanes_per_row(int64_t feat, int v) {
  int64_t need = (feat + v - 1) / v;
  int l = 1;
  while (l < need && l < kWave) l <<= 1;
  return l;
}

// Counter-based dropout mask keyed by (seed, row, col): a per-row key, then
// one 32-bit integer hash (two v_mul_lo_u32) per pair of columns, so the
// backward regenerates the forward's mask exactly.
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// Dropout seed of one launch: the caller's 64-bit value plus, when the calling
// thread has set a device seed source (sldm_set_dropout_seed_source), the word
// that pointer names, read by the kernel when it runs -- a launch recorded
// into a HIP graph then draws a new mask on every replay whose seed word the
// graph (or the host) has changed.  Host code converts a plain value at the
// first internal call; kernels take the pair and call effective_seed once.
const uint64_t* seed_source();
struct Seed {
  uint64_t value;
  const uint64_t* dev;
  Seed() = default;
  Seed(uint64_t v) : value(v), dev(seed_source()) {}
};
__device__ __forceinline__ uint64_t effective_seed(const Seed& s) {
  return s.dev ? s.value + *s.dev : s.value;
}
__device__ __forceinline__ uint32_t dropout_row_key(uint64_t seed, uint64_t row) {
  return hash32((uint32_t)seed ^ hash32((uint32_t)(seed >> 32) ^ hash32((uint32_t)row) ^
                                        (uint32_t)(row >> 32) * 0x9E3779B9u));
}
// Two columns per hash: columns 2j and 2j+1 of a row take the low and high
// 16 bits of hash32(row_key + j * golden); a column is kept iff its 16 bits
// are >= thr = round(p * 2^16), i.e. p is quantised to 2^-16 (keep-rate error
// <= 2^-17; the kept values are still scaled by the exact 1 / (1 - p)).
__device__ __forceinline__ uint32_t dropout_threshold(float p) {
  return p >= 1.f ? 65536u : (p <= 0.f ? 0u : (uint32_t)(p * 65536.f + 0.5f));
}
__device__ __forceinline__ bool dropout_keep(uint32_t row_key, uint32_t col, uint32_t thr) {
  const uint32_t h = hash32(row_key + (col >> 1) * 0x9E3779B9u);
  return ((col & 1u) ? (h >> 16) : (h & 0xFFFFu)) >= thr;
}
// Columns c, c+1 with c even: one hash.
__device__ __forceinline__ void dropout_keep2(uint32_t row_key, uint32_t c_even, uint32_t thr,
                                              bool& k0, bool& k1) {
  const uint32_t h = hash32(row_key + (c_even >> 1) * 0x9E3779B9u);
  k0 = (h & 0xFFFFu) >= thr;
  k1 = (h >> 16) >= thr;
}
// V consecutive columns from f0 (a multiple of V): pairs share a hash.
template <int V>
__device__ __forceinline__ void dropout_keepv(uint32_t row_key, uint32_t f0, uint32_t thr,
                                              bool (&keep)[V]) {
  if constexpr (V == 1) {
    keep[0] = dropout_keep(row_key, f0, thr);
  } else {
#pragma unroll
    for (int k = 0; k < V; k += 2) dropout_keep2(row_key, f0 + k, thr, keep[k], keep[k + 1]);
  }
}

// --------------------------------------------------- cross-lane reductions --
// Sum over aligned groups of G lanes (G a power of two <= 64), result in every
// lane of the group, bitwise identical across the group (each step adds a
// lane pair, a+b == b+a).  DPP / swizzle steps instead of ds_bpermute chains.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float group_sum(float v, int g) {
  if (g >= 2) v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]  (xor 1)
  if (g >= 4) v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]  (xor 2)
  if (g >= 8) v += dpp_f<0x141>(v);   // row_half_mirror      (quad <-> quad)
  if (g >= 16) v += dpp_f<0x140>(v);  // row_mirror           (half <-> half)
  if (g >= 32)                        // swap 16-lane rows inside each 32-lane half
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
  if (g >= 64)
    v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  return v;
}

// Sum over the four 16-lane rows of a wave (lanes l, l^16, l^32, l^48: an MFMA
// C-layout row's four column groups), result bitwise identical in all four:
// two gfx950 VALU lane swaps (v_permlane16_swap, v_permlane32_swap) instead of
// ds_swizzle + ds_bpermute round trips through the LDS crossbar.
__device__ __forceinline__ float row4_sum(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  const float v2 = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const uint32_t u2 = __float_as_uint(v2);
  const auto b = __builtin_amdgcn_permlane32_swap(u2, u2, false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Split-bf16 operands ("bf16x3" products): x = hi + lo with hi = bf16(x),
// lo = bf16(x - hi) (16 significant bits of fp32's 24); a product as
// a_hi b_hi + a_hi b_lo + a_lo b_hi on v_mfma_f32_16x16x32_bf16 in fp32
// accumulation is within ~2^-16 relative of the fp32 product.
typedef short bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void split_bf16x8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t ph = pack_bf16x2(v[2 * e], v[2 * e + 1]);
    h[e] = ph;
    l[e] = pack_bf16x2(v[2 * e] - bf16_lo(ph), v[2 * e + 1] - bf16_hi(ph));
  }
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}
// 4 floats -> (hi, lo) as two packed bf16x4 words (uint2 each)
__device__ __forceinline__ void split_bf16x4(const float (&v)[4], uint2& hi, uint2& lo) {
  const uint32_t h0 = pack_bf16x2(v[0], v[1]), h1 = pack_bf16x2(v[2], v[3]);
  hi = make_uint2(h0, h1);
  lo = make_uint2(pack_bf16x2(v[0] - bf16_lo(h0), v[1] - bf16_hi(h0)),
                  pack_bf16x2(v[2] - bf16_lo(h1), v[3] - bf16_hi(h1)));
}
// Three-way split ("bf16x6" products): x = hi + mid + lo exactly (3 x 8
// significand bits = fp32's 24); a product as the six partial products of
// magnitude >= 2^-18 -- lo.hi + hi.lo + mid.mid + mid.hi + hi.mid + hi.hi, small
// terms first -- on v_mfma_f32_16x16x32_bf16 with fp32 accumulation drops only
// terms below 2^-26 relative: fp32-level products at 6 x 16 MFMA cycles per
// 32-deep k-step against the exact fp32 MFMA's 8 x 32.
__device__ __forceinline__ void split3_bf16x4(const float (&v)[4], uint2& hi, uint2& mid,
                                              uint2& lo) {
  const uint32_t h0 = pack_bf16x2(v[0], v[1]), h1 = pack_bf16x2(v[2], v[3]);
  const float r0 = v[0] - bf16_lo(h0), r1 = v[1] - bf16_hi(h0);
  const float r2 = v[2] - bf16_lo(h1), r3 = v[3] - bf16_hi(h1);
  const uint32_t m0 = pack_bf16x2(r0, r1), m1 = pack_bf16x2(r2, r3);
  hi = make_uint2(h0, h1);
  mid = make_uint2(m0, m1);
  lo = make_uint2(pack_bf16x2(r0 - bf16_lo(m0), r1 - bf16_hi(m0)),
                  pack_bf16x2(r2 - bf16_lo(m1), r3 - bf16_hi(m1)));
}
__device__ __forceinline__ void split3_bf16x8(const float (&v)[8], bf16x8& hi, bf16x8& mid,
                                              bf16x8& lo) {
  const float a[4] = {v[0], v[1], v[2], v[3]}, b[4] = {v[4], v[5], v[6], v[7]};
  uint2 h0, m0, l0, h1, m1, l1;
  split3_bf16x4(a, h0, m0, l0);
  split3_bf16x4(b, h1, m1, l1);
  hi = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
  mid = __builtin_bit_cast(bf16x8, make_uint4(m0.x, m0.y, m1.x, m1.y));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
}
// One accumulator update of the six-term product (operands as MFMA fragments).
#define SLDM_MFMA_X6(acc, ah, am, al, bh, bm, bl)                                   \
  do {                                                                              \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);            \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);            \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, acc, 0, 0, 0);            \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, acc, 0, 0, 0);            \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, acc, 0, 0, 0);            \
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);            \
  } while (0)
// fp32 dense GEMMs as split-bf16 products (gemm.hip's x6 kernels; default) or
// on the exact fp32 MFMA (SLDM_FP32_GEMM=exact).
bool fp32_gemm_split();

// Big-tile bf16 dense kernels (gemm_big.hip); the gemm.hip entry points route
// conforming shapes to them.  SLDM_BIG_GEMM=0 in the environment disables them
// (A/B comparisons against the 64-row kernels).
bool big_gemm_enabled();
bool big_gemm_ok(int64_t k0, int64_t K, int64_t bn, const void* a0, int64_t lda0,
                 const void* a1, int64_t lda1, const void* b, int64_t ldb, int64_t ldo);
int big_dense_fwd(const void* a0, int64_t lda0, int64_t k0, const void* a1, int64_t lda1,
                  int64_t k1, const void* w, int64_t num_rows, int64_t nc, const float* bias,
                  const float* gamma, const float* beta, float eps, float slope, float drop_p,
                  uint64_t seed, int64_t row_off, void* out, void* xhat, float* rstd,
                  hipStream_t stream);
int big_gemm_rowscale(const void* a, int64_t lda, int64_t k, const void* b, int64_t ldb,
                      int64_t num_rows, int64_t nc, int64_t bn, const int32_t* rowptr,
                      int64_t scale_cols, void* out, int64_t ldo, void* out2, int64_t ldo2,
                      hipStream_t stream);

// Persistent register-A bf16 kernels (gemm_stream.hip) for K in {256, 512}:
// the forward at F_out = 256 and the dX GEMM at 256 | 512 output columns.
// SLDM_STREAM_GEMM=0 disables them (falls back to the big-tile kernels).
bool stream_gemm_enabled();
bool stream_dense_fwd_ok(int64_t k0, int64_t K, int64_t nc, const void* a0, int64_t lda0,
                         const void* a1, int64_t lda1, const void* w, const void* out,
                         const void* xhat, float slope);
bool stream_rowscale_ok(int64_t k, int64_t nc, const void* a, int64_t lda, const void* b,
                        int64_t ldb, const void* out, int64_t ldo, int64_t scale_cols);
int stream_dense_fwd(const void* a0, int64_t lda0, int64_t k0, const void* a1, int64_t lda1,
                     int64_t k1, const void* w, int64_t num_rows, const float* bias,
                     const float* gamma, const float* beta, float eps, float slope, float drop_p,
                     uint64_t seed, int64_t row_off, void* out, void* xhat, float* rstd,
                     hipStream_t stream);
int stream_gemm_rowscale(const void* a, int64_t lda, int64_t k, const void* b, int64_t ldb,
                         int64_t num_rows, int64_t nc, const int32_t* rowptr, int64_t scale_cols,
                         void* out, int64_t ldo, void* out2, int64_t ldo2, hipStream_t stream);
// Persistent fp32 kernels on six-term split-bf16 products (gemm_stream_f32.hip):
// the forward at F_out = 256 and the dX GEMM at 256 | 512 output columns, K in
// {256, 512}.  SLDM_STREAM_F32=0 disables them (the 64-row tile kernels run).
bool stream_f32_enabled();
bool stream_f32_dense_fwd_ok(int64_t k0, int64_t K, int64_t nc, const void* a0, int64_t lda0,
                             const void* a1, int64_t lda1, const void* w, const void* out,
                             const void* xhat);
bool stream_f32_rowscale_ok(int64_t k, int64_t nc, const void* a, int64_t lda, const void* b,
                            int64_t ldb, const void* out, int64_t ldo, const void* out2,
                            int64_t ldo2, int64_t scale_cols);
int stream_f32_dense_fwd(const void* a0, int64_t lda0, int64_t k0, const void* a1, int64_t lda1,
                         int64_t k1, const void* w, int64_t num_rows, const float* bias,
                         const float* gamma, const float* beta, float eps, float slope,
                         float drop_p, uint64_t seed, int64_t row_off, void* out, void* xhat,
                         float* rstd, hipStream_t stream);
int stream_f32_gemm_rowscale(const void* a, int64_t lda, int64_t k, const void* b, int64_t ldb,
                             int64_t num_rows, int64_t nc, const int32_t* rowptr,
                             int64_t scale_cols, void* out, int64_t ldo, void* out2, int64_t ldo2,
                             hipStream_t stream);
// gemm_ws.hip: weight-stationary dX kernel (weights in VGPRs, LDS-DMA tiles).
bool ws_gemm_enabled();
// gemm_tn_dma.hip: row-streaming dW kernel (LDS-DMA, transposed reads).
bool tn_dma_enabled();
bool tn_dma_ok(int64_t mo, int64_t n0, int64_t n1, int64_t rows, const void* a, int64_t lda,
               const void* b0, int64_t ldb0, const void* b1, int64_t ldb1);
size_t tn_dma_workspace_bytes(int64_t rows, int64_t nn);
int tn_dma(const void* a, int64_t lda, const void* b0, int64_t ldb0, const void* b1, int64_t ldb1,
           int64_t n1, int64_t rows, float* slab, int* splits_out, hipStream_t stream);
bool ws_rowscale_ok(int64_t k, int64_t nc, int64_t num_rows, const void* a, int64_t lda,
                    const void* b, int64_t ldb, const void* out, int64_t ldo, const void* out2,
                    int64_t ldo2, int64_t scale_cols);
// blk_shift > 0: the scaled half goes to ``out`` as [scale_cols >> blk_shift]
// blocks of [num_rows][1 << blk_shift] (out2 required, ldo ignored).
int ws_gemm_rowscale(const void* a, int64_t lda, int64_t k, const void* b, int64_t ldb,
                     int64_t num_rows, int64_t nc, const int32_t* rowptr, int64_t scale_cols,
                     void* out, int64_t ldo, void* out2, int64_t ldo2, hipStream_t stream,
                     int blk_shift = 0);
}  // namespace sldm

#define SLDM_REQUIRE(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      ::sldm::set_error(__VA_ARGS__);    \
      return SLDM_ERR_ARG;               \
    }                                    \
  } while (0)

#define SLDM_LAUNCH_CHECK(name)                                                   \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) {                                                       \
      ::sldm::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));   \
      return SLDM_ERR_HIP;                                                        \
    }                                                                             \
  } while (0)

#define SLDM_HIP_CHECK(expr)                                                      \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) {                                                       \
      ::sldm::set_error("%s: %s", #expr, hipGetErrorString(e_));                  \
      return SLDM_ERR_HIP;                                                        \
    }                                                                             \
  } while (0)
