// Batching of per-pack graphs resident on the GPU: the
// edge_index half of PyG's Batch.from_data_list as the reference uses it
// (main.py:166-167 DataLoader(batch_size=32) over packs loaded with
// map_location=DEVICE, dataset.py:77) -- ids offset by the running node count
// (PyG __inc__), the `batch` and `ptr` vectors -- fused with the batch's CSR
// pair, so a collated batch reaches the SageBlock with its CSR already built.
//
// One 1024-thread workgroup per graph (the graphs' edges never cross graphs,
// so each graph's CSR rows are a contiguous slice of the batch CSR):
//   1. copy + offset edge_index, write batch / ptr, validate ids, count in-
//      and out-degrees into LDS counters (ds atomics);
//   2. block scan of the counters -> the graph's rowptr / t_rowptr slice
//      (+ the graph's edge offset);
//   3. scatter local edge ids to their rows (LDS cursors, unordered);
//   4. per row, insertion-sort the edge ids (restores the original edge order
//      inside a row: the same stable order sldm_csr_build produces, so the
//      gathers sum in the same order bit for bit) and replace them by the
//      batch-global neighbour ids.
// Integer work on a few MB per batch: launch- and latency-bound, not HBM-bound.
// Three variants by LDS fit (per launch, from its largest graph): (2) the
// graph's (src, dst) pairs staged in LDS as int32 local ids while step 1
// reads them, edge ids scattered in LDS, and each slot's neighbour id written
// straight to its row position by rank (no per-row sort) -- the vehicle packs
// (~250 nodes, ~5k edges);
// (1) the same without the staged pairs (steps 3 and 5 re-read edge_index);
// (0) rows sorted in the global col / t_col slices.  Step 1 keeps kBatch
// edges' loads in flight per thread.  Measured: the global variant took 225 us per
// 32-pack batch (each row's insertion sort a chain of dependent global round
// trips), variant 1 with one load per edge per iteration 125 us.
constexpr size_t kLdsBudget = 160 * 1024;
#include "common.hpp"

namespace {

constexpr int kThreads = 1024;       // 16 waves: one workgroup per CU (LDS), latency hidden by waves
constexpr int kMaxGraphs = 48;          // per launch (kernel-argument budget)
constexpr int kMaxNodes = 16384;        // per graph: 2 x 64 KB LDS counters

struct BatchArgs {
  const int64_t* ei[kMaxGraphs];        // [2][stride] per graph
  int64_t stride[kMaxGraphs];
  int64_t ne[kMaxGraphs], eoff[kMaxGraphs];
  int32_t nn[kMaxGraphs];
  int64_t noff[kMaxGraphs];
  int64_t g0, num_graphs_total, n_total, e_total;
  int64_t* out_ei; int64_t out_ld;      // [2][out_ld]
  int64_t* batch; int64_t* ptr;
  int32_t* rowptr; int32_t* col; int32_t* t_rowptr; int32_t* t_col;
  int32_t* bad;
};

// Exclusive scan of cnt[0..n) in place (LDS), one pass over per-thread segments.
__device__ void block_exclusive_scan(int32_t* cnt, int n, int32_t* part) {
  const int t = threadIdx.x;
  const int seg = (n + kThreads - 1) / kThreads;
  const int b = min(n, t * seg), e = min(n, b + seg);
  int32_t s = 0;
  for (int i = b; i < e; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  // Hillis-Steele over the kThreads segment sums
  for (int off = 1; off < kThreads; off <<= 1) {
    const int32_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int32_t run = part[t] - s;   // exclusive prefix of this segment
  for (int i = b; i < e; ++i) {
    const int32_t c = cnt[i];
    cnt[i] = run;
    run += c;
  }
  __syncthreads();
}

// MODE 0: CSR rows sorted in global memory; 1: edge ids scattered and sorted
// in LDS; 2: as 1 with the graph's (src, dst) pairs also staged in LDS as
// int32 local ids during step 1, so steps 3 and 5 never touch global memory.
// Step 1 issues kBatch edges' loads per thread before using any of them (the
// out_ei stores may alias ei as far as the compiler knows, so a plain loop
// was one dependent global round trip per edge: ~20 per thread per phase).
constexpr int kBatch = 8;

template <int MODE>
__global__ __launch_bounds__(kThreads) void batch_graphs_kernel(BatchArgs p) {
  extern __shared__ int32_t lds[];
  const int gl = blockIdx.x;
  const int64_t g = p.g0 + gl;
  const int64_t* ei = p.ei[gl];
  const int64_t st = p.stride[gl], E = p.ne[gl], eoff = p.eoff[gl], noff = p.noff[gl];
  const int N = p.nn[gl];
  int32_t* cd = lds;                 // in-degree counters, then cursors
  int32_t* cs = lds + N;             // out-degree counters, then cursors
  int32_t* part = lds + 2 * N;       // scan scratch [kThreads]
  int32_t* ecol = part + kThreads;   // MODE >= 1: [E] dst-CSR local edge ids
  int32_t* tcol = ecol + E;          // MODE >= 1: [E] src-CSR local edge ids
  int32_t* sl = tcol + E;            // MODE 2: [E] local source ids (-1: invalid edge)
  int32_t* dl = sl + E;              // MODE 2: [E] local destination ids
  const int t = threadIdx.x;

  for (int i = t; i < 2 * N; i += kThreads) lds[i] = 0;
  for (int i = t; i < N; i += kThreads) p.batch[noff + i] = g;
  if (t == 0) {
    p.ptr[g] = noff;
    if (g == p.num_graphs_total - 1) {
      p.ptr[g + 1] = p.n_total;
      p.rowptr[p.n_total] = (int32_t)p.e_total;
      if (p.t_rowptr) p.t_rowptr[p.n_total] = (int32_t)p.e_total;
    }
  }
  __syncthreads();

  // 1. copy + offset, validate, count (kBatch edges' loads in flight per thread)
  bool bad = false;
  for (int64_t e0 = t; e0 < E; e0 += (int64_t)kThreads * kBatch) {
    int64_t s[kBatch], d[kBatch];
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      const int64_t e = min(e0 + (int64_t)u * kThreads, E - 1);   // clamped: loads unconditional
      s[u] = ei[e];
      d[u] = ei[st + e];
    }
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      const int64_t e = e0 + (int64_t)u * kThreads;
      if (e < E) {
        const bool ok = (s[u] >= 0) & (s[u] < N) & (d[u] >= 0) & (d[u] < N);
        p.out_ei[eoff + e] = s[u] + noff;
        p.out_ei[p.out_ld + eoff + e] = d[u] + noff;
        if (ok) {
          atomicAdd(&cd[d[u]], 1);
          atomicAdd(&cs[s[u]], 1);
        }
        if constexpr (MODE == 2) {
          sl[e] = ok ? (int32_t)s[u] : -1;
          dl[e] = (int32_t)d[u];
        }
        bad |= !ok;
      }
    }
  }
  if (bad) atomicOr(p.bad, 1);
  __syncthreads();

  // 2. scans -> rowptr slices
  block_exclusive_scan(cd, N, part);
  block_exclusive_scan(cs, N, part);
  for (int i = t; i < N; i += kThreads) {
    p.rowptr[noff + i] = (int32_t)(eoff + cd[i]);
    if (p.t_rowptr) p.t_rowptr[noff + i] = (int32_t)(eoff + cs[i]);
  }
  __syncthreads();

  if constexpr (MODE >= 1) {
    // 3'. scatter local edge ids into LDS, 4'. sort each row there, then the
    // neighbour ids leave in one coalesced pass
    if constexpr (MODE == 2) {
      for (int64_t e = t; e < E; e += kThreads) {
        const int32_t s = sl[e];
        if (s >= 0) {
          ecol[atomicAdd(&cd[dl[e]], 1)] = (int32_t)e;
          if (p.t_col) tcol[atomicAdd(&cs[s], 1)] = (int32_t)e;
        }
      }
    } else {
      for (int64_t e0 = t; e0 < E; e0 += (int64_t)kThreads * kBatch) {
        int64_t s[kBatch], d[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
          const int64_t e = min(e0 + (int64_t)u * kThreads, E - 1);
          s[u] = ei[e];
          d[u] = ei[st + e];
        }
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
          const int64_t e = e0 + (int64_t)u * kThreads;
          if (e < E && (s[u] >= 0) & (s[u] < N) & (d[u] >= 0) & (d[u] < N)) {
            ecol[atomicAdd(&cd[d[u]], 1)] = (int32_t)e;
            if (p.t_col) tcol[atomicAdd(&cs[s[u]], 1)] = (int32_t)e;
          }
        }
      }
    }
    __syncthreads();
    // rows past a bad id are short; those batches raise on the host anyway
    const int64_t Ev = N > 0 ? cd[N - 1] : 0;
    if constexpr (MODE == 2) {
      // 4''. no sort: each slot's edge goes to its row position by rank, the
      // number of the row's edge ids below its own (all rows in parallel, one
      // independent LDS read per comparison).  The serial per-row insertion
      // sort was the kernel's critical path: the LDS atomics of one
      // instruction hand out a row's slots in an order that can be the
      // reverse of the lanes' edge order, and a reversed row of d entries is
      // d^2 / 2 dependent LDS round trips on one thread.
      for (int dir = 0; dir < (p.t_col ? 2 : 1); ++dir) {
        const int32_t* r = dir == 0 ? ecol : tcol;
        const int32_t* cur = dir == 0 ? cd : cs;
        const int32_t* key = dir == 0 ? dl : sl;     // the edge's row
        const int32_t* nbr = dir == 0 ? sl : dl;     // its neighbour
        int32_t* outc = (dir == 0 ? p.col : p.t_col) + eoff;
        for (int64_t k = t; k < Ev; k += kThreads) {
          const int32_t e = r[k];
          const int32_t row = key[e];
          const int32_t b = row == 0 ? 0 : cur[row - 1], en = cur[row];
          int32_t rank = 0;
#pragma unroll 8
          for (int32_t j = b; j < en; ++j) rank += r[j] < e;
          outc[b + rank] = nbr[e] + (int32_t)noff;
        }
      }
      return;
    }
    for (int dir = 0; dir < (p.t_col ? 2 : 1); ++dir) {
      int32_t* r = dir == 0 ? ecol : tcol;
      const int32_t* cur = dir == 0 ? cd : cs;
      for (int i = t; i < N; i += kThreads) {
        const int32_t b = i == 0 ? 0 : cur[i - 1], e = cur[i];
        for (int32_t k = b + 1; k < e; ++k) {
          const int32_t v = r[k];
          int32_t j = k - 1;
          while (j >= b && r[j] > v) {
            r[j + 1] = r[j];
            --j;
          }
          r[j + 1] = v;
        }
      }
    }
    __syncthreads();
    for (int64_t k = t; k < Ev; k += kThreads)
      p.col[eoff + k] = (int32_t)(ei[ecol[k]] + noff);
    if (p.t_col)
      for (int64_t k = t; k < Ev; k += kThreads)
        p.t_col[eoff + k] = (int32_t)(ei[st + tcol[k]] + noff);
    return;
  }

  // 3. scatter local edge ids (order inside a row fixed in step 4)
  for (int64_t e = t; e < E; e += kThreads) {
    const int64_t s = ei[e], d = ei[st + e];
    if ((s >= 0) & (s < N) & (d >= 0) & (d < N)) {
      p.col[eoff + atomicAdd(&cd[d], 1)] = (int32_t)e;
      if (p.t_col) p.t_col[eoff + atomicAdd(&cs[s], 1)] = (int32_t)e;
    }
  }
  __syncthreads();   // workgroup-scope fence: the col / t_col writes are visible

  // 4. per row: edge ids ascending (= original order), then neighbour ids.
  // After step 3 the cursor of row i is the start of row i+1.
  for (int dir = 0; dir < (p.t_col ? 2 : 1); ++dir) {
    int32_t* c = dir == 0 ? p.col : p.t_col;
    const int32_t* cur = dir == 0 ? cd : cs;
    const int64_t nbr = dir == 0 ? 0 : st;    // dst-CSR holds sources; src-CSR destinations
    for (int i = t; i < N; i += kThreads) {
      const int32_t b = i == 0 ? 0 : cur[i - 1], e = cur[i];
      int32_t* r = c + eoff;
      for (int32_t k = b + 1; k < e; ++k) {
        const int32_t v = r[k];
        int32_t j = k - 1;
        while (j >= b && r[j] > v) {
          r[j + 1] = r[j];
          --j;
        }
        r[j + 1] = v;
      }
      for (int32_t k = b; k < e; ++k) r[k] = (int32_t)(ei[nbr + r[k]] + noff);
    }
  }
}

}  // namespace

extern "C" int sldm_batch_graphs_max_nodes(void) { return kMaxNodes; }

extern "C" int sldm_batch_graphs(int64_t num_graphs, const int64_t* const* edge_index,
                                 const int64_t* edge_row_stride, const int64_t* num_edges,
                                 const int64_t* num_nodes, int64_t* out_edge_index,
                                 int64_t out_ld, int64_t* out_batch, int64_t* out_ptr,
                                 int32_t* rowptr, int32_t* col, int32_t* t_rowptr,
                                 int32_t* t_col, int32_t* bad_index_flag, void* stream_) {
  SLDM_REQUIRE(num_graphs > 0, "sldm_batch_graphs: num_graphs must be > 0");
  SLDM_REQUIRE(edge_index && edge_row_stride && num_edges && num_nodes && out_batch && out_ptr &&
                   rowptr && bad_index_flag,
               "sldm_batch_graphs: null argument");
  SLDM_REQUIRE((t_rowptr == nullptr) == (t_col == nullptr),
               "sldm_batch_graphs: t_rowptr and t_col go together");
  int64_t n_total = 0, e_total = 0, max_n = 0, max_e = 0;
  for (int64_t g = 0; g < num_graphs; ++g) {
    SLDM_REQUIRE(num_edges[g] >= 0 && num_nodes[g] >= 0 && num_nodes[g] <= kMaxNodes,
                 "sldm_batch_graphs: graph %lld has %lld nodes (max %d) / %lld edges",
                 (long long)g, (long long)num_nodes[g], kMaxNodes, (long long)num_edges[g]);
    SLDM_REQUIRE(num_edges[g] == 0 || (edge_index[g] && edge_row_stride[g] >= num_edges[g]),
                 "sldm_batch_graphs: graph %lld: bad edge_index pointer / stride", (long long)g);
    n_total += num_nodes[g];
    e_total += num_edges[g];
    max_n = std::max<int64_t>(max_n, num_nodes[g]);
    max_e = std::max<int64_t>(max_e, num_edges[g]);
  }
  SLDM_REQUIRE(n_total < ((int64_t)1 << 31) && e_total < ((int64_t)1 << 31),
               "sldm_batch_graphs: batch too large for int32 CSR");
  SLDM_REQUIRE(out_ld >= e_total && (e_total == 0 || (out_edge_index && col)),
               "sldm_batch_graphs: output edge_index / col missing or too short");
  hipStream_t stream = sldm::as_stream(stream_);
  if (const int rc = sldm::zero_words(bad_index_flag, 1, stream); rc != SLDM_OK) return rc;
  const size_t lds_cnt = (size_t)(2 * max_n + kThreads) * sizeof(int32_t);
  const size_t lds_ids = lds_cnt + (size_t)2 * max_e * sizeof(int32_t);
  const size_t lds_stg = lds_cnt + (size_t)4 * max_e * sizeof(int32_t);
  const int mode = lds_stg <= kLdsBudget ? 2 : (lds_ids <= kLdsBudget ? 1 : 0);
  const size_t lds = mode == 2 ? lds_stg : (mode == 1 ? lds_ids : lds_cnt);
  auto kern = mode == 2 ? batch_graphs_kernel<2>
                        : (mode == 1 ? batch_graphs_kernel<1> : batch_graphs_kernel<0>);
  SLDM_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int64_t noff = 0, eoff = 0;
  for (int64_t g0 = 0; g0 < num_graphs; g0 += kMaxGraphs) {
    BatchArgs a{};
    const int cnt = (int)std::min<int64_t>(kMaxGraphs, num_graphs - g0);
    for (int k = 0; k < cnt; ++k) {
      const int64_t g = g0 + k;
      a.ei[k] = edge_index[g];
      a.stride[k] = edge_row_stride[g];
      a.ne[k] = num_edges[g];
      a.eoff[k] = eoff;
      a.nn[k] = (int32_t)num_nodes[g];
      a.noff[k] = noff;
      noff += num_nodes[g];
      eoff += num_edges[g];
    }
    a.g0 = g0; a.num_graphs_total = num_graphs; a.n_total = n_total; a.e_total = e_total;
    a.out_ei = out_edge_index; a.out_ld = out_ld;
    a.batch = out_batch; a.ptr = out_ptr;
    a.rowptr = rowptr; a.col = col; a.t_rowptr = t_rowptr; a.t_col = t_col;
    a.bad = bad_index_flag;
    kern<<<cnt, kThreads, lds, stream>>>(a);
    SLDM_LAUNCH_CHECK("batch_graphs_kernel");
  }
  return SLDM_OK;
}
