// Trajectory-radius edge construction of the vehicle graph: the O(V^2 T) pair loop of the reference's graph builders, on the GPU.
//
// Replaces gbuilder.py:85-111 (offline builder) and :241-268
// (GraphOnlineCreator, the latency path of rcv.py:77):
//   for i, for j != i (in this order):
//     d = ||x[i,:,0:2] - x[j,:,0:2]||_2 per frame        (numpy, float32)
//     d = d[(p[i] > 0.5) & (p[j] > 0.5)]                  (frames both present)
//     if d.size and d.min() <= radius:
//        edge (i, j), attr [d.min(), d.max(), d.mean(), (d**2).mean()]
// Arithmetic is numpy's float32 arithmetic, reproduced exactly: the norm as
// sqrt(dx*dx + dy*dy) with no contraction, mean/msq through numpy's pairwise
// summation (8 strided accumulators per <= 128-element block, halves split at
// multiples of 8 above that) and one float32 division; radius compared in
// float32 (numpy 2 promotion of a Python float against float32).  Edges come
// out i-major, j ascending -- the reference's list order.
//
// One thread per ordered pair; the pair's distances of the frames both
// vehicles are present in are compacted into a private array (T <= kMaxT),
// then reduced.  Pass 1 writes a keep flag and the four stats per pair, an
// exclusive scan (hipcub) turns flags into edge slots, pass 2 scatters.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

// numpy does not fuse: every product and sum below rounds on its own, through
// the *_rn helpers whose bodies switch contraction off (HIP's own __f*_rn are
// plain operators in a header where it stays on), and sqrtf is the correctly
// rounded square root (__fsqrt_rn is the approximate native one in this HIP
// build).

namespace {

constexpr int kBlock = 256;
constexpr int kMaxT = 256;   // frames per pack (the reference's packs: 100)

// numpy/_core/src/umath/loops_utils.h.src pairwise_sum, float32 accumulators:
// < 8 elements sequentially from 0; <= 128 with 8 strided accumulators then
// the tail; longer: halves split at a multiple of 8.  Recursion unrolled at
// compile time (D levels: n <= 128 * 2^D).
// IEEE single operations that never fuse (contract(off) in their bodies).
__device__ __forceinline__ float add_rn(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float sub_rn(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}
__device__ __forceinline__ float mul_rn(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float div_rn(float a, float b) {
#pragma clang fp contract(off)
  return a / b;
}

template <bool SQ>
__device__ __forceinline__ float elem(const float* a, int i) {
#pragma clang fp contract(off)
  return SQ ? mul_rn(a[i], a[i]) : a[i];
}

template <bool SQ>
__device__ float block_sum(const float* a, int n) {
#pragma clang fp contract(off)
  if (n < 8) {
    float res = 0.f;
    for (int i = 0; i < n; ++i) res = add_rn(res, elem<SQ>(a, i));
    return res;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = elem<SQ>(a, j);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = add_rn(r[j], elem<SQ>(a, i + j));
  }
  float res = add_rn(add_rn(add_rn(r[0], r[1]), add_rn(r[2], r[3])),
                        add_rn(add_rn(r[4], r[5]), add_rn(r[6], r[7])));
  for (; i < n; ++i) res = add_rn(res, elem<SQ>(a, i));
  return res;
}

template <bool SQ, int D>
__device__ float pairwise_sum(const float* a, int n) {
#pragma clang fp contract(off)
  if constexpr (D == 0) {
    return block_sum<SQ>(a, n);
  } else {
    if (n <= 128) return block_sum<SQ>(a, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return add_rn(pairwise_sum<SQ, D - 1>(a, n2), pairwise_sum<SQ, D - 1>(a + n2, n - n2));
  }
}

__global__ __launch_bounds__(kBlock) void radius_pairs_kernel(
    const float* __restrict__ pos, int64_t pos_sv, int64_t pos_st, int64_t pos_sc,
    const float* __restrict__ pres, int64_t pres_sv, int64_t pres_st, int nv, int nt,
    float radius, int32_t* __restrict__ keep, float4* __restrict__ stats) {
#pragma clang fp contract(off)
  const int64_t pair = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (pair >= (int64_t)nv * nv) return;
  const int i = (int)(pair / nv), j = (int)(pair % nv);
  int k = 0;
  float mn = 0.f, mx = 0.f;
  float d[kMaxT];
  if (i != j) {
    for (int t = 0; t < nt; ++t) {
      const bool both = pres[i * pres_sv + t * pres_st] > 0.5f && pres[j * pres_sv + t * pres_st] > 0.5f;
      if (!both) continue;
      const float dx = sub_rn(pos[i * pos_sv + t * pos_st], pos[j * pos_sv + t * pos_st]);
      const float dy = sub_rn(pos[i * pos_sv + t * pos_st + pos_sc],
                                 pos[j * pos_sv + t * pos_st + pos_sc]);
      const float v = sqrtf(add_rn(mul_rn(dx, dx), mul_rn(dy, dy)));
      mn = k == 0 ? v : fminf(mn, v);
      mx = k == 0 ? v : fmaxf(mx, v);
      d[k++] = v;
    }
  }
  const bool kept = k > 0 && mn <= radius;
  keep[pair] = kept ? 1 : 0;
  if (kept) {
    const float fk = (float)k;
    stats[pair] = make_float4(mn, mx, div_rn(pairwise_sum<false, 2>(d, k), fk),
                              div_rn(pairwise_sum<true, 2>(d, k), fk));
  }
}

__global__ __launch_bounds__(kBlock) void radius_emit_kernel(
    const int32_t* __restrict__ keep, const int32_t* __restrict__ slot,
    const float4* __restrict__ stats, int nv, int64_t* __restrict__ edge_index, int64_t cap,
    float4* __restrict__ edge_attr, int32_t* __restrict__ num_edges) {
  const int64_t pair = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t npairs = (int64_t)nv * nv;
  if (pair >= npairs) return;
  if (pair == npairs - 1) *num_edges = slot[pair] + keep[pair];
  if (!keep[pair]) return;
  const int64_t e = slot[pair];
  edge_index[e] = pair / nv;          // row 0: source i
  edge_index[cap + e] = pair % nv;    // row 1: target j
  edge_attr[e] = stats[pair];
}

}  // namespace

extern "C" size_t sldm_radius_edges_workspace_bytes(int64_t num_vehicles) {
  const int64_t np = num_vehicles > 0 ? num_vehicles * num_vehicles : 1;
  size_t scan = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const int32_t*)nullptr,
                                         (int32_t*)nullptr, (int)np);
  return (size_t)np * (4 + 4 + 16) + scan + 4 * 256;
}

extern "C" int sldm_radius_edges(const float* pos, int64_t pos_sv, int64_t pos_st, int64_t pos_sc,
                                 const float* presence, int64_t pres_sv, int64_t pres_st,
                                 int64_t num_vehicles, int64_t num_frames, float radius,
                                 int64_t* edge_index, int64_t capacity, float* edge_attr,
                                 int32_t* num_edges, void* workspace, size_t workspace_bytes,
                                 void* stream_) {
  SLDM_REQUIRE(num_vehicles >= 0 && num_frames >= 0 && num_frames <= kMaxT,
               "sldm_radius_edges: frames %lld outside [0, %d]", (long long)num_frames, kMaxT);
  SLDM_REQUIRE(num_vehicles * num_vehicles < ((int64_t)1 << 31),
               "sldm_radius_edges: too many vehicles (%lld)", (long long)num_vehicles);
  SLDM_REQUIRE(num_edges, "sldm_radius_edges: NULL num_edges");
  hipStream_t stream = sldm::as_stream(stream_);
  if (num_vehicles == 0) {
    return sldm::zero_words(num_edges, 1, stream);
  }
  SLDM_REQUIRE(pos && presence && edge_index && edge_attr,
               "sldm_radius_edges: NULL argument");
  SLDM_REQUIRE(capacity >= num_vehicles * (num_vehicles - 1),
               "sldm_radius_edges: capacity %lld < V(V-1)", (long long)capacity);
  const size_t need = sldm_radius_edges_workspace_bytes(num_vehicles);
  SLDM_REQUIRE(workspace && workspace_bytes >= need,
               "sldm_radius_edges: workspace too small (%zu < %zu)", workspace_bytes, need);
  const int64_t np = num_vehicles * num_vehicles;
  auto al = [](uintptr_t p) { return (p + 255) & ~(uintptr_t)255; };
  int32_t* keep = reinterpret_cast<int32_t*>(al(reinterpret_cast<uintptr_t>(workspace)));
  int32_t* slot = reinterpret_cast<int32_t*>(al(reinterpret_cast<uintptr_t>(keep + np)));
  float4* stats = reinterpret_cast<float4*>(al(reinterpret_cast<uintptr_t>(slot + np)));
  void* scan_tmp = reinterpret_cast<void*>(al(reinterpret_cast<uintptr_t>(stats + np)));
  size_t scan_bytes = workspace_bytes - (reinterpret_cast<char*>(scan_tmp) -
                                         reinterpret_cast<char*>(workspace));
  const unsigned grid = (unsigned)((np + kBlock - 1) / kBlock);
  radius_pairs_kernel<<<grid, kBlock, 0, stream>>>(pos, pos_sv, pos_st, pos_sc, presence, pres_sv,
                                                   pres_st, (int)num_vehicles, (int)num_frames,
                                                   radius, keep, stats);
  SLDM_LAUNCH_CHECK("radius_pairs_kernel");
  SLDM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, keep, slot, (int)np,
                                                  stream));
  radius_emit_kernel<<<grid, kBlock, 0, stream>>>(keep, slot, stats, (int)num_vehicles,
                                                  edge_index, capacity,
                                                  reinterpret_cast<float4*>(edge_attr), num_edges);
  SLDM_LAUNCH_CHECK("radius_emit_kernel");
  return SLDM_OK;
}
