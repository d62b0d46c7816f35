// Streaming ceilings for the dense kernels' byte mixes (diagnostic):
// NR input streams read, NW output streams written, each 5.12 GB (10M rows x
// 512 B), 16-B vectors, grid-stride over a resident grid.  The forward kernel
// is 2R:2W, dX 1R:2W, dW 3R:0W.
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int NR, int NW, int U>
__global__ __launch_bounds__(256) void rw(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                          const uint4* __restrict__ c, uint4* __restrict__ o,
                                          uint4* __restrict__ p, int64_t n, uint4* sink) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int64_t i0 = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += stride) {
    uint4 v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * 256;
      if (i < n) {
        v[u][0] = a[i];
        if (NR > 1) v[u][1] = b[i];
        if (NR > 2) v[u][2] = c[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * 256;
      if (i >= n) continue;
      uint4 s = v[u][0];
      if (NR > 1) { s.x ^= v[u][1].x; s.y ^= v[u][1].y; s.z ^= v[u][1].z; s.w ^= v[u][1].w; }
      if (NR > 2) { s.x ^= v[u][2].x; s.y ^= v[u][2].y; s.z ^= v[u][2].z; s.w ^= v[u][2].w; }
      if (NW > 0) o[i] = s;
      if (NW > 1) p[i] = make_uint4(s.y, s.x, s.w, s.z);
      if (NW == 0) { acc.x ^= s.x; acc.y ^= s.y; acc.z ^= s.z; acc.w ^= s.w; }
    }
  }
  if (NW == 0 && acc.x == 0x12345678u) sink[0] = acc;
}

template <int NR, int NW, int U>
int run(uint4* bufs[5], int64_t n, int grid, const char* name) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 2; ++it)
    rw<NR, NW, U><<<grid, 256>>>(bufs[0], bufs[1], bufs[2], bufs[3], bufs[4], n, bufs[4]);
  CK(hipEventRecord(e0));
  const int reps = 5;
  for (int it = 0; it < reps; ++it)
    rw<NR, NW, U><<<grid, 256>>>(bufs[0], bufs[1], bufs[2], bufs[3], bufs[4], n, bufs[4]);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = (double)(NR + NW) * n * 16;
  printf("%-10s grid %6d U %d: %.3f ms  %.0f GB/s\n", name, grid, U, ms, bytes / ms / 1e6);
  return 0;
}

// Low-occupancy read-only stream (one 512-thread block per CU, like the GEMM
// stream kernels): D loads of 16 B in flight per lane.  STRIDED = the stream
// kernels' MFMA-fragment pattern: per instruction 16 rows x 64 B (lane = row
// r16, 16-B chunk q), successive instructions walk the row's 64-B pieces;
// otherwise each instruction reads 1 KB contiguous.
template <bool STRIDED, int D>
__global__ __launch_bounds__(512) void rd(const uint4* __restrict__ a, int64_t rows, uint4* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t groups = rows / 16;                 // 16-row groups (8 KB)
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int64_t g = (int64_t)blockIdx.x * 8 + wave; g < groups; g += (int64_t)gridDim.x * 8) {
    const uint4* base = a + g * 512;                // 16 rows x 32 vectors
    uint4 v[32];
#pragma unroll
    for (int s0 = 0; s0 < 8; s0 += D / 1) {
#pragma unroll
      for (int s = s0; s < s0 + D && s < 8; ++s) {
        const int idx = STRIDED ? (lane & 15) * 32 + s * 4 + (lane >> 4) : s * 64 + lane;
        v[s] = base[idx];
      }
#pragma unroll
      for (int s = s0; s < s0 + D && s < 8; ++s) {
        acc.x ^= v[s].x; acc.y ^= v[s].y; acc.z ^= v[s].z; acc.w ^= v[s].w;
      }
    }
  }
  if (acc.x == 0x12345678u) sink[0] = acc;
}

template <bool STRIDED, int D>
int run_rd(const uint4* a, int64_t rows, int grid, uint4* sink, const char* name) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  rd<STRIDED, D><<<grid, 512>>>(a, rows, sink);
  CK(hipEventRecord(e0));
  for (int it = 0; it < 5; ++it) rd<STRIDED, D><<<grid, 512>>>(a, rows, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  printf("%-22s grid %5d D %d: %.3f ms  %.0f GB/s\n", name, grid, D, ms, rows * 512.0 / ms / 1e6);
  return 0;
}

// The dX stream kernel's memory pattern without the MFMAs: per wave 32 rows
// (2 x 16-row slabs), 8 k-steps of strided 64-B loads per slab with a ring of
// D steps, then an epilogue burst of 2 x 8 strided 16-B stores per slab into
// each of two [rows][256] outputs (the paired-tile store layout).
template <int D, bool CR, bool FL>
__global__ __launch_bounds__(512) void dxpat(const uint4* __restrict__ a, uint4* __restrict__ o1,
                                             uint4* __restrict__ o2, int64_t rows, uint4* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int64_t groups = rows / 32;
  for (int64_t g = (int64_t)blockIdx.x * 8 + wave; g < groups; g += (int64_t)gridDim.x * 8) {
    const uint4* base = a + g * 1024;
    uint4 acc[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
#pragma unroll
    for (int s0 = 0; s0 < 8; s0 += D) {
      uint4 v[D][2];
#pragma unroll
      for (int s = 0; s < D; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m)
          v[s][m] = CR ? base[(m * D + s) * 64 + lane] : base[(16 * m + r16) * 32 + (s0 + s) * 4 + q];
#pragma unroll
      for (int s = 0; s < D; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          acc[m].x += v[s][m].x; acc[m].y ^= v[s][m].y; acc[m].z += v[s][m].z; acc[m].w ^= v[s][m].w;
        }
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int64_t row = g * 32 + 16 * m + r16;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (FL) {   // 2 full 512-B rows per instruction
          const int64_t rr = g * 32 + 16 * m + 2 * t + (lane >> 5);
          o1[rr * 32 + (lane & 31)] = acc[m];
          o2[rr * 32 + (lane & 31)] = make_uint4(acc[m].y, acc[m].x, acc[m].w, acc[m].z);
        } else {
          const int c = 4 * t + ((q & 1) ? 2 + (q - 1) / 2 : q / 2);   // 16-B column index
          o1[row * 32 + c] = acc[m];
          o2[row * 32 + c] = make_uint4(acc[m].y, acc[m].x, acc[m].w, acc[m].z);
        }
      }
    }
  }
}

template <int D, bool CR, bool FL>
int run_dx(uint4* bufs[5], int64_t rows, int grid) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  dxpat<D, CR, FL><<<grid, 512>>>(bufs[1], bufs[2], bufs[3], rows, bufs[4]);
  CK(hipEventRecord(e0));
  for (int it = 0; it < 5; ++it)
    dxpat<D, CR, FL><<<grid, 512>>>(bufs[1], bufs[2], bufs[3], rows, bufs[4]);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  printf("dX pattern (no MFMA) reads %s stores %s grid %5d D %d: %.3f ms  %.0f GB/s\n",
         CR ? "contig" : "strided", FL ? "rows  " : "64B   ", grid, D, ms,
         rows * 1536.0 / ms / 1e6);
  return 0;
}

int main() {
  const int64_t n = 10000000LL * 512 / 16;   // 16-B vectors per stream
  uint4* bufs[5];
  for (int i = 0; i < 5; ++i) {
    const int64_t sz = i == 0 ? 3 * n * 16 : n * 16;
    CK(hipMalloc(&bufs[i], sz));
    CK(hipMemset(bufs[i], i, sz));
  }
  for (int rep = 0; rep < 2; ++rep) {
    run_dx<4, false, false>(bufs, 10000000, 256);
    run_dx<4, true, false>(bufs, 10000000, 256);
    run_dx<4, false, true>(bufs, 10000000, 256);
    run_dx<4, true, true>(bufs, 10000000, 256);
  }
  if (getenv("PROBE_DX_ONLY")) return 0;
  const int64_t rows = 30000000;   // 15.4 GB: the three dY/agg/h streams of dW
  for (int grid : {256}) {
    run_rd<true, 4>(bufs[0], rows, grid, bufs[4], "read strided 64B");
    run_rd<false, 4>(bufs[0], rows, grid, bufs[4], "read contiguous");
    run_rd<true, 8>(bufs[0], rows, grid, bufs[4], "read strided 64B");
    run_rd<false, 8>(bufs[0], rows, grid, bufs[4], "read contiguous");
    run_rd<true, 2>(bufs[0], rows, grid, bufs[4], "read strided 64B");
    run_rd<false, 2>(bufs[0], rows, grid, bufs[4], "read contiguous");
  }
  for (int grid : {1024, 8192}) {
    run<2, 2, 2>(bufs, n, grid, "fwd 2R2W");
    run<1, 2, 2>(bufs, n, grid, "dX 1R2W");
    run<3, 0, 2>(bufs, n, grid, "dW 3R0W");
    run<1, 1, 2>(bufs, n, grid, "copy 1R1W");
    run<2, 2, 4>(bufs, n, grid, "fwd 2R2W");
    run<1, 2, 4>(bufs, n, grid, "dX 1R2W");
    run<3, 0, 4>(bufs, n, grid, "dW 3R0W");
  }
  return 0;
}
