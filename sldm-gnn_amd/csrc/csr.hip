// CSR build for the SageBlock hot path.
//
// edge_index [2,E] (int64 or int32, row 0 = source j, row 1 = target i; the
// layout produced by /root/reference/src/gbuilder.py:85-112 and batched by PyG
// collate) -> CSR by destination (rowptr, col) and CSR by source (t_rowptr,
// t_col).  Both are a STABLE sort of the edges by key, so inside a row the
// entries keep the original edge order — the order in which PyG's CPU
// scatter_add_ accumulates (oracle/csr_ref.c states the same contract in C).
//
// Integer work, HBM-bound: one pass to narrow/validate ids to int32, an LSD
// radix sort (rocPRIM, stable) on ceil(log2 (N+1)) key bits, and one pass that
// turns the sorted keys into row pointers without atomics.  An edge (N, N) is
// padding (fixed-shape edge_index buffers of captured graphs): its key N sorts
// behind row N-1, past rowptr[N], where no kernel reads.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

namespace {

constexpr int kBlock = 256;

template <typename TIdx>
__global__ __launch_bounds__(kBlock) void narrow_validate_kernel(
    const TIdx* __restrict__ ei, int64_t E, int64_t N, uint32_t* __restrict__ src32,
    uint32_t* __restrict__ dst32, int32_t* __restrict__ bad) {
  int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= E) return;
  int64_t s = (int64_t)ei[e];
  int64_t d = (int64_t)ei[E + e];
  // (N, N) is a padding edge: it keeps key N and sorts behind every row
  bool ok = ((s >= 0) & (s < N) & (d >= 0) & (d < N)) | ((s == N) & (d == N));
  if (!ok) {
    atomicOr(bad, 1);
    s = 0;
    d = 0;
  }
  src32[e] = (uint32_t)s;
  dst32[e] = (uint32_t)d;
}

// rowptr[k] = first position p with key[p] >= k, for k in [0, N].
// Thread p fills the keys in (key[p-1], key[p]] — O(E + N) total, no atomics.
__global__ __launch_bounds__(kBlock) void rowptr_from_sorted_kernel(
    const uint32_t* __restrict__ keys, int64_t E, int64_t N, int32_t* __restrict__ rowptr) {
  int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p > E) return;
  int64_t prev = (p == 0) ? -1 : (int64_t)keys[p - 1];
  int64_t cur = (p == E) ? N : (int64_t)keys[p];
  for (int64_t k = prev + 1; k <= cur; ++k) rowptr[k] = (int32_t)p;
}

__global__ __launch_bounds__(kBlock) void degree_iota_kernel(const int32_t* __restrict__ rowptr,
                                                             int64_t N, uint32_t* __restrict__ deg,
                                                             uint32_t* __restrict__ ids) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= N) return;
  deg[i] = (uint32_t)(rowptr[i + 1] - rowptr[i]);
  ids[i] = (uint32_t)i;
}

unsigned key_bits(int64_t N) {
  unsigned bits = 0;
  while (bits < 32 && ((int64_t)1 << bits) < N) ++bits;
  return bits == 0 ? 1 : bits;
}

size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

size_t sort_temp_bytes(int64_t E, int64_t N) {
  size_t bytes = 0;
  if (E == 0) return 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)E, 0u,
                                  key_bits(N + 1), (hipStream_t)0);
  return bytes;
}

}  // namespace

// ------------------------------------------------------------------------
// Longest-first row schedule for skewed (power-law) graphs: order = rows by
// decreasing degree (stable).  The gather kernels walk rows in this order, so
// hub rows start first and the rows sharing a wave have similar lengths;
// every row is still summed sequentially in CSR order.
namespace {
size_t order_temp_bytes(int64_t N) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs_desc(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)N,
                                       0u, 32u, (hipStream_t)0);
  return bytes;
}
}  // namespace

extern "C" size_t sldm_degree_order_workspace_bytes(int64_t num_nodes) {
  if (num_nodes <= 0) return 256;
  return 3 * align_up(sizeof(uint32_t) * (size_t)num_nodes) + align_up(order_temp_bytes(num_nodes)) + 256;
}

extern "C" int sldm_degree_order(const int32_t* rowptr, int64_t num_nodes, int32_t* order,
                                 void* workspace, size_t workspace_bytes, void* stream_) {
  const int64_t N = num_nodes;
  SLDM_REQUIRE(N >= 0 && N < ((int64_t)1 << 31), "sldm_degree_order: bad N=%lld", (long long)N);
  if (N == 0) return SLDM_OK;
  SLDM_REQUIRE(rowptr && order, "sldm_degree_order: NULL argument");
  const size_t need = sldm_degree_order_workspace_bytes(N);
  SLDM_REQUIRE(workspace && workspace_bytes >= need,
               "sldm_degree_order: workspace too small (%zu < %zu)", workspace_bytes, need);
  hipStream_t stream = sldm::as_stream(stream_);
  char* ws = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(workspace) + 255) & ~(uintptr_t)255);
  const size_t arr = align_up(sizeof(uint32_t) * (size_t)N);
  uint32_t* deg = reinterpret_cast<uint32_t*>(ws);
  uint32_t* ids = reinterpret_cast<uint32_t*>(ws + arr);
  uint32_t* deg_out = reinterpret_cast<uint32_t*>(ws + 2 * arr);
  void* temp = ws + 3 * arr;
  size_t temp_bytes = order_temp_bytes(N);
  degree_iota_kernel<<<(unsigned)((N + kBlock - 1) / kBlock), kBlock, 0, stream>>>(rowptr, N, deg, ids);
  SLDM_LAUNCH_CHECK("degree_iota_kernel");
  SLDM_HIP_CHECK(rocprim::radix_sort_pairs_desc(temp, temp_bytes, (const uint32_t*)deg, deg_out,
                                                (const uint32_t*)ids,
                                                reinterpret_cast<uint32_t*>(order), (size_t)N,
                                                0u, 32u, stream));
  return SLDM_OK;
}

extern "C" size_t sldm_csr_workspace_bytes(int64_t num_edges, int64_t num_nodes) {
  if (num_edges < 0 || num_nodes < 0) return 0;
  size_t arr = align_up(sizeof(uint32_t) * (size_t)(num_edges > 0 ? num_edges : 1));
  return 3 * arr + align_up(sort_temp_bytes(num_edges, num_nodes)) + 256;
}

extern "C" int sldm_csr_build(const void* edge_index, int index_is_int64, int64_t num_edges,
                              int64_t num_nodes, int32_t* rowptr, int32_t* col,
                              int32_t* t_rowptr, int32_t* t_col, int32_t* bad_index_flag,
                              void* workspace, size_t workspace_bytes, void* stream_) {
  const int64_t E = num_edges, N = num_nodes;
  SLDM_REQUIRE(E >= 0 && N >= 0, "sldm_csr_build: negative size (E=%lld, N=%lld)",
               (long long)E, (long long)N);
  SLDM_REQUIRE(E < ((int64_t)1 << 31) && N < ((int64_t)1 << 31),
               "sldm_csr_build: E=%lld / N=%lld exceed the int32 CSR limit", (long long)E,
               (long long)N);
  SLDM_REQUIRE(rowptr != nullptr && bad_index_flag != nullptr,
               "sldm_csr_build: rowptr / bad_index_flag must not be NULL");
  SLDM_REQUIRE(E == 0 || (t_rowptr == nullptr) == (t_col == nullptr),
               "sldm_csr_build: t_rowptr and t_col must both be set or both NULL");
  hipStream_t stream = sldm::as_stream(stream_);

  if (E == 0) {
    int rc = sldm::zero_words(rowptr, (size_t)(N + 1), stream);
    if (rc == SLDM_OK && t_rowptr) rc = sldm::zero_words(t_rowptr, (size_t)(N + 1), stream);
    return rc;
  }
  SLDM_REQUIRE(edge_index != nullptr && col != nullptr,
               "sldm_csr_build: edge_index / col must not be NULL");
  SLDM_REQUIRE(N > 0, "sldm_csr_build: E=%lld edges on an empty node set", (long long)E);
  const size_t need = sldm_csr_workspace_bytes(E, N);
  SLDM_REQUIRE(workspace != nullptr && workspace_bytes >= need,
               "sldm_csr_build: workspace too small (%zu < %zu bytes)", workspace_bytes, need);

  char* ws = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(workspace) + 255) & ~(uintptr_t)255);
  const size_t arr = align_up(sizeof(uint32_t) * (size_t)E);
  uint32_t* src32 = reinterpret_cast<uint32_t*>(ws);
  uint32_t* dst32 = reinterpret_cast<uint32_t*>(ws + arr);
  uint32_t* keys_out = reinterpret_cast<uint32_t*>(ws + 2 * arr);
  void* temp = ws + 3 * arr;
  size_t temp_bytes = sort_temp_bytes(E, N);
  const unsigned bits = key_bits(N + 1);    // keys in [0, N]: N marks padding edges

  const unsigned grid_e = (unsigned)((E + kBlock - 1) / kBlock);
  if (index_is_int64)
    narrow_validate_kernel<int64_t><<<grid_e, kBlock, 0, stream>>>(
        reinterpret_cast<const int64_t*>(edge_index), E, N, src32, dst32, bad_index_flag);
  else
    narrow_validate_kernel<int32_t><<<grid_e, kBlock, 0, stream>>>(
        reinterpret_cast<const int32_t*>(edge_index), E, N, src32, dst32, bad_index_flag);
  SLDM_LAUNCH_CHECK("narrow_validate_kernel");

  const unsigned grid_p = (unsigned)((E + 1 + kBlock - 1) / kBlock);
  // By destination: keys = dst, values = src  ->  col.
  SLDM_HIP_CHECK(rocprim::radix_sort_pairs(temp, temp_bytes, (const uint32_t*)dst32, keys_out,
                                           (const uint32_t*)src32,
                                           reinterpret_cast<uint32_t*>(col), (size_t)E, 0u, bits,
                                           stream));
  rowptr_from_sorted_kernel<<<grid_p, kBlock, 0, stream>>>(keys_out, E, N, rowptr);
  SLDM_LAUNCH_CHECK("rowptr_from_sorted_kernel");
  if (t_rowptr) {
    // By source: keys = src, values = dst  ->  t_col.
    SLDM_HIP_CHECK(rocprim::radix_sort_pairs(temp, temp_bytes, (const uint32_t*)src32, keys_out,
                                             (const uint32_t*)dst32,
                                             reinterpret_cast<uint32_t*>(t_col), (size_t)E, 0u,
                                             bits, stream));
    rowptr_from_sorted_kernel<<<grid_p, kBlock, 0, stream>>>(keys_out, E, N, t_rowptr);
    SLDM_LAUNCH_CHECK("rowptr_from_sorted_kernel(t)");
  }
  return SLDM_OK;
}
