// CSR row gather: the SageBlock neighbour aggregation
// and its transpose for the backward (A8).
//
// Replaces, per SAGEConv call (sageblock.py:18 -> PyG 2.7.0 propagate):
//   x_j = x.index_select(0, edge_index[0])              [E,F] message tensor
//   agg = scatter_add_(dst, x_j) / count.clamp(min=1)   MeanAggregation
// without materialising the [E,F] messages: each destination row is summed
// straight from the source rows it names.
//
// Layout / mapping (HBM-bound; algorithmic bytes per call
//   B = E*(4 + F*s) + (N+1)*4 + N*F*s_out [+ N*F*s_add]):
//   - a row is owned by LPR lanes (power of two, <= one wave64); each lane
//     holds V consecutive features (16 B: 4 fp32 or 8 bf16) per chunk, NCH
//     chunks per lane when a row is wider than a wave's 1 KiB;
//   - every source row is read as whole 16-B-per-lane vectors: a bf16 F=256
//     row is 512 B = one coalesced half-wave load; two rows share a wave;
//   - up to 8 source rows per row-group are in flight before the first
//     accumulate (batches of 8/4/2/1, no per-element predication, so the
//     compiler keeps the loads un-waited);
//   - tables >= 1 GiB: output rows stored non-temporal (sldm::store_vec,
//     nt_gather in common.hpp; source-row loads stay cached);
//   - fp32 accumulation in CSR order -> bit-identical to the reference's CPU
//     scatter_add_ for fp32 input; the mean divides by the fp32 degree
//     (PyG divides by the fp32 count).
//
// High-degree rows (power-law graphs, BASELINE C5: in-degree up to ~10^4)
// are split ("hub plan", sldm_gather_rows_split): one row group would sum a
// 10^4-edge row serially (~1250 dependent batches), so the launch puts the
// hubs' fixed-length edge chunks in its FIRST slots -- each chunk summed by
// its own row group, in CSR order, into an fp32 partial row of a workspace --
// and the ordinary rows after them in natural order, skipping every row with
// degree > max_deg.  A second, tiny kernel adds each hub's chunk partials in
// chunk order (deterministic; within fp32 reassociation of the CPU order),
// divides by the degree, adds the addend and stores the row.
#include "common.hpp"

#include <mutex>

namespace {

constexpr int kBlock = 256;

// Hub plan of one launch (all zero / INT32_MAX: no split).
struct HubArgs {
  const int32_t* chunk_row;   // [num_chunks] hub row of chunk c
  const int32_t* chunk_beg;   // [num_chunks] first CSR position of chunk c
  int64_t num_chunks;
  int chunk_len;              // edges per chunk (the last chunk of a row may be shorter)
  int max_deg;                // rows with degree > max_deg are hubs (skipped by the row slots)
  float* partials;            // [num_chunks, feat] fp32
};

template <typename TI, typename TO, int V, int NCH, bool MEAN, bool ADD, int NT>
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(
    const TI* __restrict__ x, int64_t ldx, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const int32_t* __restrict__ order, int64_t nrows,
    int feat, int lpr_log2,
    const TO* __restrict__ addend, int64_t lda, TO* __restrict__ out, int64_t ldo, HubArgs hub) {
  const int lpr = 1 << lpr_log2;
  const int lane_in_row = threadIdx.x & (lpr - 1);
  const int64_t slot = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lpr_log2;
  // slots [0, num_chunks): hub chunks; then one slot per ordinary row
  const bool chunk = slot < hub.num_chunks;
  const int64_t ridx = slot - hub.num_chunks;
  if (!chunk && ridx >= nrows) return;
  // Optional row schedule / subset: slot ridx handles row order[ridx].
  const int64_t row = chunk ? (int64_t)hub.chunk_row[slot] : (order ? (int64_t)order[ridx] : ridx);

  int f0[NCH];
  bool act[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    int f = (lane_in_row + c * lpr) * V;
    act[c] = f < feat;
    f0[c] = act[c] ? f : feat - V;  // clamp: inactive lanes re-read a valid vector
  }

  float acc[NCH][V];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[c][v] = 0.0f;

  int beg, end;
  if (chunk) {
    beg = hub.chunk_beg[slot];
    const int row_end = rowptr[row + 1];
    end = row_end - beg > hub.chunk_len ? beg + hub.chunk_len : row_end;
  } else {
    beg = rowptr[row];
    end = rowptr[row + 1];
    if (end - beg > hub.max_deg) return;     // a hub: summed by its chunk slots
  }

  // The addend row (root-path gradient) is independent of the neighbour
  // loads: issue it first so it is in flight with them instead of costing
  // one more dependent memory round trip after the last batch.
  float a[NCH][V];
  if constexpr (ADD) {
    if (!chunk) {
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        sldm::load_vec<TO, V, sldm::kStreamOperandsNt && (NT & 1) != 0>(addend + row * lda + f0[c],
                                                                         a[c]);
    }
  }

  // Column indices one batch ahead: the next 8 are loaded (clamped to the
  // row) before the current batch's rows are summed, so the index load of
  // batch b+1 overlaps the row loads of batch b instead of following them.
  auto load_idx = [&](int k, int (&dst)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) dst[u] = col[k + u < end ? k + u : end - 1];
  };
  auto batch = [&](const int* idx, auto u_const) {
    constexpr int U = decltype(u_const)::value;
    float d[U][NCH][V];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        sldm::load_vec<TI, V, (NT & 2) != 0>(x + (int64_t)idx[u] * ldx + f0[c], d[u][c]);
    return [&, d]() mutable {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < NCH; ++c)
#pragma unroll
          for (int v = 0; v < V; ++v) acc[c][v] += d[u][c][v];
    };
  };

  int k = beg;
  if (k < end) {
    int idx[8];
    load_idx(k, idx);
    for (; k + 8 <= end; k += 8) {
      auto sum = batch(idx, std::integral_constant<int, 8>{});
      if (k + 8 < end) load_idx(k + 8, idx);
      sum();
    }
    // tail (< 8 left): indices already in idx[0 .. end-k)
    const int left = end - k;
    int o = 0;
    if (left & 4) { batch(idx, std::integral_constant<int, 4>{})(); o = 4; }
    if (left & 2) { batch(idx + o, std::integral_constant<int, 2>{})(); o += 2; }
    if (left & 1) batch(idx + o, std::integral_constant<int, 1>{})();
  }

  if (chunk) {                                // fp32 partial of this chunk
    float* pp = hub.partials + slot * (int64_t)feat;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (!act[c]) continue;
#pragma unroll
      for (int v = 0; v < V; v += 4 < V ? 4 : V) {
        if constexpr (V >= 4) sldm::Vec<float, 4>::store(pp + f0[c] + v, acc[c] + v);
        else sldm::Vec<float, V>::store(pp + f0[c] + v, acc[c] + v);
      }
    }
    return;
  }
  if (MEAN) {
    const float cnt = (float)(end - beg > 0 ? end - beg : 1);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[c][v] = acc[c][v] / cnt;
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (!act[c]) continue;
    if constexpr (ADD) {
#pragma unroll
      for (int v = 0; v < V; ++v) acc[c][v] = a[c][v] + acc[c][v];
    }
    sldm::store_vec<TO, V, (NT & 1) != 0>(out + row * ldo + f0[c], acc[c]);
  }
}

// Second pass of the hub split: row group h adds hub h's chunk partials in
// chunk order, then mean / addend / store exactly as the row slots do.
template <typename TO, int V, int NCH, bool MEAN, bool ADD>
__global__ __launch_bounds__(kBlock) void gather_hub_finish_kernel(
    const float* __restrict__ partials, const int32_t* __restrict__ hub_rows,
    const int32_t* __restrict__ hub_chunk_ptr, int64_t num_hubs, const int32_t* __restrict__ rowptr,
    int feat, int lpr_log2, const TO* __restrict__ addend, int64_t lda, TO* __restrict__ out,
    int64_t ldo) {
  const int lpr = 1 << lpr_log2;
  const int lane_in_row = threadIdx.x & (lpr - 1);
  const int64_t h = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> lpr_log2;
  if (h >= num_hubs) return;
  const int64_t row = hub_rows[h];
  const int c0 = hub_chunk_ptr[h], c1 = hub_chunk_ptr[h + 1];
  int f0[NCH];
  bool act[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int f = (lane_in_row + c * lpr) * V;
    act[c] = f < feat;
    f0[c] = act[c] ? f : feat - V;
  }
  float acc[NCH][V];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[c][v] = 0.f;
  for (int k = c0; k < c1; ++k) {
    const float* pp = partials + (int64_t)k * feat;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[c][v] += pp[f0[c] + v];
  }
  if (MEAN) {
    const int deg = rowptr[row + 1] - rowptr[row];
    const float cnt = (float)(deg > 0 ? deg : 1);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[c][v] = acc[c][v] / cnt;
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (!act[c]) continue;
    if constexpr (ADD) {
      float a[V];
      sldm::Vec<TO, V>::load(addend + row * lda + f0[c], a);
#pragma unroll
      for (int v = 0; v < V; ++v) acc[c][v] = a[v] + acc[c][v];
    }
    sldm::Vec<TO, V>::store(out + row * ldo + f0[c], acc[c]);
  }
}

// Hub plan of one call (host side): the HubArgs plus the finish kernel's
// hub list.
struct HubPlan {
  HubArgs k;
  const int32_t* hub_rows;
  const int32_t* hub_chunk_ptr;
  int64_t num_hubs;
};

template <typename TI, typename TO, int V, bool MEAN, bool ADD>
int launch_nch(const TI* x, int64_t ldx, const int32_t* rowptr, const int32_t* col, const int32_t* order,
               int64_t nrows, int feat, const TO* addend, int64_t lda, TO* out, int64_t ldo,
               const HubPlan& hp, hipStream_t stream) {
  int lpr = sldm::lanes_per_row(feat, V);
  int lpr_log2 = 0;
  while ((1 << lpr_log2) < lpr) ++lpr_log2;
  const int64_t nch = (feat + (int64_t)lpr * V - 1) / ((int64_t)lpr * V);
  const int64_t threads = (nrows + hp.k.num_chunks) << lpr_log2;
  const int64_t grid = (threads + kBlock - 1) / kBlock;
  SLDM_REQUIRE(grid < ((int64_t)1 << 31), "sldm_gather_rows: grid too large");
  const int nt = sldm::nt_gather(nrows * ldx * (int64_t)sizeof(TI));
#define SLDM_GATHER_LAUNCH(NC, NTV)                                                           \
  gather_rows_kernel<TI, TO, V, NC, MEAN, ADD, NTV><<<(unsigned)grid, kBlock, 0, stream>>>(  \
      x, ldx, rowptr, col, order, nrows, feat, lpr_log2, addend, lda, out, ldo, hp.k)
#define SLDM_HUB_FINISH(NC)                                                                  \
  if (hp.num_hubs > 0)                                                                       \
    gather_hub_finish_kernel<TO, V, NC, MEAN, ADD>                                           \
        <<<(unsigned)(((hp.num_hubs << lpr_log2) + kBlock - 1) / kBlock), kBlock, 0, stream>>>( \
            hp.k.partials, hp.hub_rows, hp.hub_chunk_ptr, hp.num_hubs, rowptr, feat, lpr_log2, \
            addend, lda, out, ldo)
#define SLDM_GATHER_CASE(NC)                                                                 \
  case NC:                                                                                   \
    if (nt == 3) SLDM_GATHER_LAUNCH(NC, 3);                                                  \
    else if (nt == 1) SLDM_GATHER_LAUNCH(NC, 1);                                             \
    else SLDM_GATHER_LAUNCH(NC, 0);                                                          \
    SLDM_HUB_FINISH(NC);                                                                     \
    break;
  switch (nch) {
    SLDM_GATHER_CASE(1)
    SLDM_GATHER_CASE(2)
    SLDM_GATHER_CASE(3)
    SLDM_GATHER_CASE(4)
    default:
      sldm::set_error("sldm_gather_rows: feat=%d too wide (max %d)", feat, 4 * 64 * V);
      return SLDM_ERR_ARG;
  }
#undef SLDM_GATHER_CASE
#undef SLDM_HUB_FINISH
#undef SLDM_GATHER_LAUNCH
  SLDM_LAUNCH_CHECK("gather_rows_kernel");
  return SLDM_OK;
}

template <typename TI, typename TO, bool MEAN, bool ADD>
int launch_vec(int v, const void* x, int64_t ldx, const int32_t* rowptr, const int32_t* col, const int32_t* order,
               int64_t nrows, int feat, const void* addend, int64_t lda, void* out, int64_t ldo,
               const HubPlan& hp, hipStream_t stream) {
  auto xi = reinterpret_cast<const TI*>(x);
  auto ad = reinterpret_cast<const TO*>(addend);
  auto o = reinterpret_cast<TO*>(out);
  switch (v) {
    case 8:
      if constexpr (sizeof(TI) == 2 && sizeof(TO) == 2)
        return launch_nch<TI, TO, 8, MEAN, ADD>(xi, ldx, rowptr, col, order, nrows, feat, ad, lda, o, ldo, hp, stream);
      break;
    case 4:
      return launch_nch<TI, TO, 4, MEAN, ADD>(xi, ldx, rowptr, col, order, nrows, feat, ad, lda, o, ldo, hp, stream);
    case 2:
      return launch_nch<TI, TO, 2, MEAN, ADD>(xi, ldx, rowptr, col, order, nrows, feat, ad, lda, o, ldo, hp, stream);
    case 1:
      return launch_nch<TI, TO, 1, MEAN, ADD>(xi, ldx, rowptr, col, order, nrows, feat, ad, lda, o, ldo, hp, stream);
  }
  sldm::set_error("sldm_gather_rows: unsupported vector width %d", v);
  return SLDM_ERR_ARG;
}

template <typename T, bool MEAN, bool ADD>
int dispatch_same(const void* x, int64_t ldx, const int32_t* rowptr, const int32_t* col, const int32_t* order,
                  int64_t nrows, int feat, const void* addend, int64_t lda, void* out,
                  int64_t ldo, const HubPlan& hp, hipStream_t stream) {
  int v = sldm::pick_vec((int)sizeof(T), feat, {ldx, ldo, ADD ? lda : (int64_t)0},
                         {x, out, addend});
  return launch_vec<T, T, MEAN, ADD>(v, x, ldx, rowptr, col, order, nrows, feat, addend, lda, out, ldo,
                                     hp, stream);
}

}  // namespace

namespace {
int gather_rows_impl(int x_dtype, const void* x, int64_t ldx, const int32_t* rowptr,
                     const int32_t* col, const int32_t* row_order, int64_t num_rows, int64_t feat,
                     int mean, const void* addend, int64_t ld_add, int out_dtype, void* out,
                     int64_t ldo, const HubPlan& hp, void* stream_) {
  SLDM_REQUIRE(x_dtype == out_dtype && (x_dtype == SLDM_F32 || x_dtype == SLDM_BF16),
               "sldm_gather_rows: dtypes (%d -> %d) unsupported: both F32 or both BF16",
               x_dtype, out_dtype);
  SLDM_REQUIRE(num_rows >= 0 && feat >= 0 && feat < (1 << 20),
               "sldm_gather_rows: bad sizes rows=%lld feat=%lld", (long long)num_rows,
               (long long)feat);
  if ((num_rows == 0 && hp.k.num_chunks == 0) || feat == 0) return SLDM_OK;
  SLDM_REQUIRE(x && rowptr && col && out, "sldm_gather_rows: NULL pointer argument");
  SLDM_REQUIRE(ldx >= feat && ldo >= feat && (!addend || ld_add >= feat),
               "sldm_gather_rows: leading dimension smaller than feat");
  hipStream_t stream = sldm::as_stream(stream_);
  const int f = (int)feat;
  const bool add = addend != nullptr;
  if (x_dtype == SLDM_F32) {
    if (mean)
      return add ? dispatch_same<float, true, true>(x, ldx, rowptr, col, row_order, num_rows, f, addend, ld_add, out, ldo, hp, stream)
                 : dispatch_same<float, true, false>(x, ldx, rowptr, col, row_order, num_rows, f, addend, ld_add, out, ldo, hp, stream);
    return add ? dispatch_same<float, false, true>(x, ldx, rowptr, col, row_order, num_rows, f, addend, ld_add, out, ldo, hp, stream)
               : dispatch_same<float, false, false>(x, ldx, rowptr, col, row_order, num_rows, f, addend, ld_add, out, ldo, hp, stream);
  }
  if (mean)
    return add ? dispatch_same<uint16_t, true, true>(x, ldx, rowptr, col, row_order, num_rows, f, addend, ld_add, out, ldo, hp, stream)
               : dispatch_same<uint16_t, true, false>(x, ldx, rowptr, col, row_order, num_rows, f, addend, ld_add, out, ldo, hp, stream);
  return add ? dispatch_same<uint16_t, false, true>(x, ldx, rowptr, col, row_order, num_rows, f, addend, ld_add, out, ldo, hp, stream)
             : dispatch_same<uint16_t, false, false>(x, ldx, rowptr, col, row_order, num_rows, f, addend, ld_add, out, ldo, hp, stream);
}
}  // namespace

extern "C" int sldm_gather_rows(int x_dtype, const void* x, int64_t ldx, const int32_t* rowptr,
                                const int32_t* col, const int32_t* row_order,
                                int64_t num_rows, int64_t feat, int mean,
                                const void* addend, int64_t ld_add, int out_dtype, void* out,
                                int64_t ldo, void* stream_) {
  HubPlan hp{{nullptr, nullptr, 0, 1, INT32_MAX, nullptr}, nullptr, nullptr, 0};
  return gather_rows_impl(x_dtype, x, ldx, rowptr, col, row_order, num_rows, feat, mean, addend,
                          ld_add, out_dtype, out, ldo, hp, stream_);
}

extern "C" int sldm_gather_rows_split(int x_dtype, const void* x, int64_t ldx,
                                      const int32_t* rowptr, const int32_t* col,
                                      const int32_t* row_order, int64_t num_rows, int64_t feat,
                                      int mean, const void* addend, int64_t ld_add, int out_dtype,
                                      void* out, int64_t ldo, const int32_t* hub_rows,
                                      const int32_t* hub_chunk_ptr, int64_t num_hubs,
                                      const int32_t* chunk_row, const int32_t* chunk_beg,
                                      int64_t num_chunks, int32_t chunk_len, int32_t max_deg,
                                      float* partials, void* stream_) {
  SLDM_REQUIRE(num_hubs >= 0 && num_chunks >= 0 && chunk_len >= 1 && max_deg >= 0,
               "sldm_gather_rows_split: bad hub plan (hubs %lld, chunks %lld, len %d, max %d)",
               (long long)num_hubs, (long long)num_chunks, chunk_len, max_deg);
  SLDM_REQUIRE((num_chunks == 0) == (num_hubs == 0), "sldm_gather_rows_split: hubs without chunks");
  SLDM_REQUIRE(num_hubs == 0 || (hub_rows && hub_chunk_ptr && chunk_row && chunk_beg && partials),
               "sldm_gather_rows_split: NULL hub plan argument");
  HubPlan hp{{chunk_row, chunk_beg, num_chunks, chunk_len, max_deg, partials}, hub_rows,
             hub_chunk_ptr, num_hubs};
  return gather_rows_impl(x_dtype, x, ldx, rowptr, col, row_order, num_rows, feat, mean, addend,
                          ld_add, out_dtype, out, ldo, hp, stream_);
}

// ------------------------------------------------ no-allocation variant --
// sldm_gather_rows_split for callers that cannot allocate device memory (code
// under HIP graph capture, tight serving loops): the chunk partials live in
// `scratch`, a file-scope device array of kStaticPartialFloats floats that each
// GPU the library runs on holds until the process ends.  Host code never
// passes the array's name to a kernel (on the host it is only a stand-in for
// the symbol): the device address comes from hipGetSymbolAddress, once per
// device with that device current, and is kept per device.
namespace {
constexpr size_t kStaticPartialFloats = (size_t)4 << 20;          // 16 MiB
static __device__ __align__(256) float scratch[kStaticPartialFloats];
constexpr int kMaxDevices = 64;
float* g_scratch_ptr[kMaxDevices] = {};
std::mutex g_scratch_mu;

// Device address of `scratch` on the current device (resolved on first use).
int static_partials(float** out) {
  int dev = -1;
  SLDM_HIP_CHECK(hipGetDevice(&dev));
  SLDM_REQUIRE(dev >= 0 && dev < kMaxDevices, "sldm_gather_rows_split_static: device %d", dev);
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  if (!g_scratch_ptr[dev]) {
    float* p = nullptr;
    SLDM_HIP_CHECK(hipGetSymbolAddress(reinterpret_cast<void**>(&p), HIP_SYMBOL(scratch)));
    SLDM_REQUIRE(p != nullptr, "sldm_gather_rows_split_static: no device address for the scratch");
    g_scratch_ptr[dev] = p;
  }
  *out = g_scratch_ptr[dev];
  return SLDM_OK;
}
}  // namespace

extern "C" size_t sldm_gather_rows_split_static_max_floats(void) { return kStaticPartialFloats; }

extern "C" int sldm_gather_rows_split_static(
    int x_dtype, const void* x, int64_t ldx, const int32_t* rowptr, const int32_t* col,
    const int32_t* row_order, int64_t num_rows, int64_t feat, int mean, const void* addend,
    int64_t ld_add, int out_dtype, void* out, int64_t ldo, const int32_t* hub_rows,
    const int32_t* hub_chunk_ptr, int64_t num_hubs, const int32_t* chunk_row,
    const int32_t* chunk_beg, int64_t num_chunks, int32_t chunk_len, int32_t max_deg,
    void* stream_) {
  SLDM_REQUIRE(num_chunks >= 0 && feat >= 0 &&
                   (feat == 0 || (uint64_t)num_chunks <= kStaticPartialFloats / (uint64_t)feat),
               "sldm_gather_rows_split_static: %lld chunks x %lld features exceed the static "
               "scratch of %zu floats; use sldm_gather_rows_split with a caller workspace",
               (long long)num_chunks, (long long)feat, kStaticPartialFloats);
  float* partials = nullptr;
  if (num_chunks > 0) {
    const int rc = static_partials(&partials);
    if (rc != SLDM_OK) return rc;
  }
  // every chunk slot of the launch overwrites its whole partial row before the
  // finish kernel reads it, so nothing of the previous call's contents is read
  return sldm_gather_rows_split(x_dtype, x, ldx, rowptr, col, row_order, num_rows, feat, mean,
                                addend, ld_add, out_dtype, out, ldo, hub_rows, hub_chunk_ptr,
                                num_hubs, chunk_row, chunk_beg, num_chunks, chunk_len, max_deg,
                                partials, stream_);
}

// ------------------------------------------------------------------------
namespace {
template <typename T, int V>
__global__ __launch_bounds__(kBlock) void scale_inv_deg_kernel(T* __restrict__ d, int64_t ld,
                                                               const int32_t* __restrict__ rowptr,
                                                               int64_t nrows, int feat) {
  const int64_t vecs_per_row = feat / V;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= nrows * vecs_per_row) return;
  const int64_t row = i / vecs_per_row;
  const int64_t f = (i - row * vecs_per_row) * V;
  const int deg = rowptr[row + 1] - rowptr[row];
  const float cnt = (float)(deg > 0 ? deg : 1);
  float r[V];
  sldm::Vec<T, V>::load(d + row * ld + f, r);
#pragma unroll
  for (int v = 0; v < V; ++v) r[v] = r[v] / cnt;
  sldm::Vec<T, V>::store(d + row * ld + f, r);
}

template <typename T>
int launch_scale(void* d, int64_t ld, const int32_t* rowptr, int64_t nrows, int feat,
                 hipStream_t stream) {
  int v = sldm::pick_vec((int)sizeof(T), feat, {ld}, {d});
  auto p = reinterpret_cast<T*>(d);
  const int64_t n = nrows * (feat / v);
  const unsigned grid = (unsigned)((n + kBlock - 1) / kBlock);
  switch (v) {
    case 8:
      if constexpr (sizeof(T) == 2) scale_inv_deg_kernel<T, 8><<<grid, kBlock, 0, stream>>>(p, ld, rowptr, nrows, feat);
      break;
    case 4: scale_inv_deg_kernel<T, 4><<<grid, kBlock, 0, stream>>>(p, ld, rowptr, nrows, feat); break;
    case 2: scale_inv_deg_kernel<T, 2><<<grid, kBlock, 0, stream>>>(p, ld, rowptr, nrows, feat); break;
    default: scale_inv_deg_kernel<T, 1><<<grid, kBlock, 0, stream>>>(p, ld, rowptr, nrows, feat); break;
  }
  SLDM_LAUNCH_CHECK("scale_inv_deg_kernel");
  return SLDM_OK;
}
}  // namespace

extern "C" int sldm_scale_rows_by_inv_deg(int dtype, void* d, int64_t ld, const int32_t* rowptr,
                                          int64_t num_rows, int64_t feat, void* stream_) {
  SLDM_REQUIRE(dtype == SLDM_F32 || dtype == SLDM_BF16, "sldm_scale_rows_by_inv_deg: dtype %d",
               dtype);
  if (num_rows <= 0 || feat <= 0) return SLDM_OK;
  SLDM_REQUIRE(d && rowptr && ld >= feat, "sldm_scale_rows_by_inv_deg: bad arguments");
  hipStream_t stream = sldm::as_stream(stream_);
  return dtype == SLDM_F32 ? launch_scale<float>(d, ld, rowptr, num_rows, (int)feat, stream)
                           : launch_scale<uint16_t>(d, ld, rowptr, num_rows, (int)feat, stream);
}
