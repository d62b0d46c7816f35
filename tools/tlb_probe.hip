// Probe: does the random-row gather rate depend on how the 5 GB feature table
// is mapped (TLB reach)?  Standalone: hipcc --offload-arch=gfx950 -O3
// tools/tlb_probe.hip -o /tmp/tlb_probe && /tmp/tlb_probe
//
// Same access pattern as the SageBlock forward gather at C4 (10M rows of
// 512 B, 100M uniform random in-edges, 32 lanes x 16 B per row, 8 rows in
// flight), over tables allocated as:
//   default     hipMalloc
//   contiguous  hipExtMallocWithFlags(hipDeviceMallocContiguous)
//   aligned1g   hipMalloc(size + 1 GiB), base rounded up to 1 GiB
// and, for reference, a 0.6 GB table (1.25M rows).  Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void gather(const uint4* __restrict__ x, const int* __restrict__ rowptr,
                                              const int* __restrict__ col, int64_t nrows,
                                              uint4* __restrict__ out) {
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 5;
  const int l = threadIdx.x & 31;
  if (row >= nrows) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int k = rowptr[row];
  const int end = rowptr[row + 1];
  auto add = [&](uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[2 * i] += __uint_as_float(w[i] << 16);
      acc[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
    }
  };
  for (; k + 8 <= end; k += 8) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = x[(int64_t)col[k + u] * 32 + l];
#pragma unroll
    for (int u = 0; u < 8; ++u) add(v[u]);
  }
  for (; k < end; ++k) add(x[(int64_t)col[k] * 32 + l]);
  uint4 o;
  o.x = (__float_as_uint(acc[0]) >> 16) | (__float_as_uint(acc[1]) & 0xffff0000u);
  o.y = (__float_as_uint(acc[2]) >> 16) | (__float_as_uint(acc[3]) & 0xffff0000u);
  o.z = (__float_as_uint(acc[4]) >> 16) | (__float_as_uint(acc[5]) & 0xffff0000u);
  o.w = (__float_as_uint(acc[6]) >> 16) | (__float_as_uint(acc[7]) & 0xffff0000u);
  out[row * 32 + l] = o;
}

static float run(const char* name, uint4* x, int64_t ntab, const int* rowptr, const int* col,
                 int64_t nrows, int64_t e, uint4* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned grid = (unsigned)((nrows * 32 + 255) / 256);
  for (int i = 0; i < 2; ++i) gather<<<grid, 256>>>(x, rowptr, col, nrows, out);
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int i = 0; i < reps; ++i) gather<<<grid, 256>>>(x, rowptr, col, nrows, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double bytes = (double)e * (512 + 4) + (double)nrows * 512 + (nrows + 1) * 4.0;
  printf("%-12s table=%6.2f GB base=%p  %8.3f ms  %7.1f GB/s\n", name, ntab * 512 / 1e9,
         (void*)x, ms, bytes / ms / 1e6);
  return ms;
}

int main() {
  const int64_t n = 10000000, e = 100000000;
  // uniform random CSR: dst-sorted, per-row counts from random dst
  std::vector<int> rowptr(n + 1, 0), col(e);
  std::mt19937_64 rng(1);
  std::vector<int> dst(e);
  for (int64_t i = 0; i < e; ++i) dst[i] = (int)(rng() % n);
  for (int64_t i = 0; i < e; ++i) rowptr[dst[i] + 1]++;
  for (int64_t i = 0; i < n; ++i) rowptr[i + 1] += rowptr[i];
  std::vector<int> fill(rowptr.begin(), rowptr.end() - 1);
  for (int64_t i = 0; i < e; ++i) col[fill[dst[i]]++] = (int)(rng() % n);
  int *d_rowptr, *d_col, *d_col_small;
  CK(hipMalloc(&d_rowptr, (n + 1) * 4));
  CK(hipMalloc(&d_col, e * 4));
  CK(hipMemcpy(d_rowptr, rowptr.data(), (n + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_col, col.data(), e * 4, hipMemcpyHostToDevice));
  std::vector<int> col_small(e);
  for (int64_t i = 0; i < e; ++i) col_small[i] = col[i] % 1250000;
  CK(hipMalloc(&d_col_small, e * 4));
  CK(hipMemcpy(d_col_small, col_small.data(), e * 4, hipMemcpyHostToDevice));
  uint4* out;
  CK(hipMalloc(&out, n * 512));
  const size_t tb = (size_t)n * 512;

  uint4* x0;
  CK(hipMalloc(&x0, tb));
  CK(hipMemset(x0, 0x3c, tb));
  run("default", x0, n, d_rowptr, d_col, n, e, out);
  run("small0.6GB", x0, 1250000, d_rowptr, d_col_small, n, e, out);
  CK(hipFree(x0));

  uint4* x1 = nullptr;
  hipError_t err = hipExtMallocWithFlags((void**)&x1, tb, hipDeviceMallocContiguous);
  if (err == hipSuccess) {
    CK(hipMemset(x1, 0x3c, tb));
    run("contiguous", x1, n, d_rowptr, d_col, n, e, out);
    CK(hipFree(x1));
  } else {
    printf("contiguous   alloc failed: %s\n", hipGetErrorString(err));
    (void)hipGetLastError();
  }

  char* raw;
  const size_t G = 1ull << 30;
  CK(hipMalloc(&raw, tb + G));
  uint4* x2 = (uint4*)(((uintptr_t)raw + G - 1) & ~(uintptr_t)(G - 1));
  CK(hipMemset(x2, 0x3c, tb));
  run("aligned1g", x2, n, d_rowptr, d_col, n, e, out);
  CK(hipFree(raw));

  char* raw2;
  CK(hipExtMallocWithFlags((void**)&raw2, tb + G, hipDeviceMallocContiguous));
  uint4* x3 = (uint4*)(((uintptr_t)raw2 + G - 1) & ~(uintptr_t)(G - 1));
  CK(hipMemset(x3, 0x3c, tb));
  run("contig+1g", x3, n, d_rowptr, d_col, n, e, out);
  CK(hipFree(raw2));
  return 0;
}
