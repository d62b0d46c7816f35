// A non-Python host of libsldm_sage.so: the C ABI (include/sldm_sage.h) driven
// from plain C++ with the HIP runtime -- what a host in another language binds
// through its FFI.  Builds the CSR of a random graph
// on the GPU, runs the mean aggregation (the reference's index_select +
// scatter-mean, sageblock.py:18) and its transpose-gather backward, and checks
// both bit for bit against a host restatement of the reference's order (fp32
// sums in edge order, one bf16 rounding).  Then the same three launches are
// recorded into a HIP graph (up to 2^20 edges) and replayed on new edge lists
// whose tail is padding -- edges (N, N), which the build ignores -- and a
// LayerNorm + dropout launch is recorded with a device seed word: replays
// with different words drop different masks, and a replay equals the eager
// launch whose seed is value + word.  Exit status 0 on success.
//   usage: abi_host [num_nodes num_edges feat]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sldm_sage.h"

#define HIP_OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) {                        \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)
#define SLDM_CALL(x) do { int rc_ = (x); if (rc_ != SLDM_OK) {                              \
  std::fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, sldm_last_error()); return 3; } } while (0)

static uint64_t lcg(uint64_t& s) { s = s * 6364136223846793005ull + 1442695040888963407ull; return s >> 33; }
static float bf2f(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; std::memcpy(&f, &u, 4); return f; }
static uint16_t f2bf(float f) {   // round to nearest even (finite inputs)
  uint32_t u; std::memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// out[i] = (add[i] +) sum over CSR row i of x[col[k]] (/ max(1, deg) if mean)
static void host_gather(const std::vector<int32_t>& rp, const std::vector<int32_t>& col,
                        const std::vector<uint16_t>& x, const std::vector<uint16_t>* add, int F,
                        bool mean, std::vector<uint16_t>& out) {
  const int n = (int)rp.size() - 1;
  out.assign((size_t)n * F, 0);
  std::vector<float> acc(F);
  for (int i = 0; i < n; ++i) {
    std::fill(acc.begin(), acc.end(), 0.f);
    for (int k = rp[i]; k < rp[i + 1]; ++k)
      for (int f = 0; f < F; ++f) acc[f] += bf2f(x[(size_t)col[k] * F + f]);
    const float cnt = (float)(rp[i + 1] - rp[i] > 0 ? rp[i + 1] - rp[i] : 1);
    for (int f = 0; f < F; ++f) {
      float v = mean ? acc[f] / cnt : acc[f];
      if (add) v = bf2f((*add)[(size_t)i * F + f]) + v;
      out[(size_t)i * F + f] = f2bf(v);
    }
  }
}

// stable counting sort of edges by key -> (rowptr, other endpoint)
static void host_csr(const std::vector<int64_t>& ei, int64_t E, int n, bool by_dst,
                     std::vector<int32_t>& rp, std::vector<int32_t>& col) {
  rp.assign(n + 1, 0);
  col.assign(E, 0);
  for (int64_t e = 0; e < E; ++e) ++rp[ei[(by_dst ? E : 0) + e] + 1];
  for (int i = 0; i < n; ++i) rp[i + 1] += rp[i];
  std::vector<int32_t> fill(rp.begin(), rp.end() - 1);
  for (int64_t e = 0; e < E; ++e)
    col[fill[ei[(by_dst ? E : 0) + e]]++] = (int32_t)ei[(by_dst ? 0 : E) + e];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 5000;
  const int64_t E = argc > 2 ? std::atoll(argv[2]) : 40000;
  const int F = argc > 3 ? std::atoi(argv[3]) : 256;
  if (sldm_abi_version() != SLDM_ABI_VERSION) {
    std::fprintf(stderr, "ABI %d != %d\n", sldm_abi_version(), SLDM_ABI_VERSION);
    return 4;
  }
  uint64_t seed = 12345;
  std::vector<int64_t> ei(2 * E);
  for (auto& v : ei) v = (int64_t)(lcg(seed) % (uint64_t)n);
  std::vector<uint16_t> x((size_t)n * F), add((size_t)n * F);
  for (auto& v : x) v = f2bf(((float)(lcg(seed) % 20001) - 10000.f) / 4096.f);
  for (auto& v : add) v = f2bf(((float)(lcg(seed) % 20001) - 10000.f) / 4096.f);

  hipStream_t st;
  HIP_OK(hipStreamCreate(&st));
  int64_t* d_ei; uint16_t *d_x, *d_add, *d_out, *d_dx; int32_t *d_rp, *d_col, *d_trp, *d_tcol, *d_bad;
  void* d_ws;
  const size_t ws = sldm_csr_workspace_bytes(E, n);
  HIP_OK(hipMalloc(&d_ei, sizeof(int64_t) * 2 * (E > 0 ? E : 1)));
  HIP_OK(hipMalloc(&d_x, sizeof(uint16_t) * x.size()));
  HIP_OK(hipMalloc(&d_add, sizeof(uint16_t) * add.size()));
  HIP_OK(hipMalloc(&d_out, sizeof(uint16_t) * x.size()));
  HIP_OK(hipMalloc(&d_dx, sizeof(uint16_t) * x.size()));
  HIP_OK(hipMalloc(&d_rp, sizeof(int32_t) * (n + 1)));
  HIP_OK(hipMalloc(&d_trp, sizeof(int32_t) * (n + 1)));
  // (at least one element: the ABI takes no NULL index arrays, even for E = 0)
  HIP_OK(hipMalloc(&d_col, sizeof(int32_t) * (E > 0 ? E : 1)));
  HIP_OK(hipMalloc(&d_tcol, sizeof(int32_t) * (E > 0 ? E : 1)));
  HIP_OK(hipMalloc(&d_bad, sizeof(int32_t)));
  HIP_OK(hipMalloc(&d_ws, ws));
  if (E) HIP_OK(hipMemcpy(d_ei, ei.data(), sizeof(int64_t) * 2 * E, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_x, x.data(), sizeof(uint16_t) * x.size(), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_add, add.data(), sizeof(uint16_t) * add.size(), hipMemcpyHostToDevice));
  HIP_OK(hipMemset(d_bad, 0, sizeof(int32_t)));

  SLDM_CALL(sldm_csr_build(d_ei, 1, E, n, d_rp, d_col, d_trp, d_tcol, d_bad, d_ws, ws, st));
  // forward: mean aggregation; backward: transpose sum + root-path addend
  SLDM_CALL(sldm_gather_rows(SLDM_BF16, d_x, F, d_rp, d_col, nullptr, n, F, 1, nullptr, 0,
                             SLDM_BF16, d_out, F, st));
  SLDM_CALL(sldm_gather_rows(SLDM_BF16, d_x, F, d_trp, d_tcol, nullptr, n, F, 0, d_add, F,
                             SLDM_BF16, d_dx, F, st));
  HIP_OK(hipStreamSynchronize(st));

  int32_t bad = 0;
  std::vector<int32_t> rp(n + 1), col(E), trp(n + 1), tcol(E);
  std::vector<uint16_t> out(x.size()), dx(x.size());
  HIP_OK(hipMemcpy(&bad, d_bad, sizeof(int32_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(rp.data(), d_rp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
  if (E) HIP_OK(hipMemcpy(col.data(), d_col, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(trp.data(), d_trp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
  if (E) HIP_OK(hipMemcpy(tcol.data(), d_tcol, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(out.data(), d_out, sizeof(uint16_t) * out.size(), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(dx.data(), d_dx, sizeof(uint16_t) * dx.size(), hipMemcpyDeviceToHost));

  std::vector<int32_t> hrp, hcol, htrp, htcol;
  host_csr(ei, E, n, true, hrp, hcol);
  host_csr(ei, E, n, false, htrp, htcol);
  std::vector<uint16_t> hout, hdx;
  host_gather(hrp, hcol, x, nullptr, F, true, hout);
  host_gather(htrp, htcol, x, &add, F, false, hdx);
  const bool ok = bad == 0 && rp == hrp && col == hcol && trp == htrp && tcol == htcol &&
                  out == hout && dx == hdx;
  std::printf("abi_host: N=%d E=%lld F=%d csr %s, mean gather %s, transpose gather %s\n", n,
              (long long)E, F, (rp == hrp && col == hcol && trp == htrp && tcol == htcol) ? "equal" : "DIFFERS",
              out == hout ? "bit-exact" : "DIFFERS", dx == hdx ? "bit-exact" : "DIFFERS");
  bool cap_ok = true, drop_ok = true;
  if (E > 0 && E <= ((int64_t)1 << 20)) {
    // ---- CSR build + both gathers as one captured graph, replayed on new edges ----
    hipGraph_t graph;
    hipGraphExec_t exec;
    HIP_OK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    SLDM_CALL(sldm_csr_build(d_ei, 1, E, n, d_rp, d_col, d_trp, d_tcol, d_bad, d_ws, ws, st));
    SLDM_CALL(sldm_gather_rows(SLDM_BF16, d_x, F, d_rp, d_col, nullptr, n, F, 1, nullptr, 0,
                               SLDM_BF16, d_out, F, st));
    SLDM_CALL(sldm_gather_rows(SLDM_BF16, d_x, F, d_trp, d_tcol, nullptr, n, F, 0, d_add, F,
                               SLDM_BF16, d_dx, F, st));
    HIP_OK(hipStreamEndCapture(st, &graph));
    HIP_OK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3 && cap_ok; ++rep) {
      const int64_t real = rep == 1 ? E / 3 : E - E / 8;       // the rest of the buffer is padding
      std::vector<int64_t> padded(2 * E, (int64_t)n), re(2 * real);
      for (int64_t e = 0; e < real; ++e) {
        re[e] = padded[e] = (int64_t)(lcg(seed) % (uint64_t)n);
        re[real + e] = padded[E + e] = (int64_t)(lcg(seed) % (uint64_t)n);
      }
      HIP_OK(hipMemcpy(d_ei, padded.data(), sizeof(int64_t) * 2 * E, hipMemcpyHostToDevice));
      // the program's own eager work between replays
      SLDM_CALL(sldm_gather_rows(SLDM_BF16, d_add, F, d_rp, d_col, nullptr, n, F, 1, nullptr, 0,
                                 SLDM_BF16, d_out, F, st));
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipGraphLaunch(exec, st));
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipMemcpy(&bad, d_bad, sizeof(int32_t), hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(rp.data(), d_rp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(col.data(), d_col, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(trp.data(), d_trp, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(tcol.data(), d_tcol, sizeof(int32_t) * E, hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(out.data(), d_out, sizeof(uint16_t) * out.size(), hipMemcpyDeviceToHost));
      HIP_OK(hipMemcpy(dx.data(), d_dx, sizeof(uint16_t) * dx.size(), hipMemcpyDeviceToHost));
      host_csr(re, real, n, true, hrp, hcol);
      host_csr(re, real, n, false, htrp, htcol);
      host_gather(hrp, hcol, x, nullptr, F, true, hout);
      host_gather(htrp, htcol, x, &add, F, false, hdx);
      col.resize(real);
      tcol.resize(real);
      cap_ok = bad == 0 && rp == hrp && col == hcol && trp == htrp && tcol == htcol &&
               out == hout && dx == hdx;
      col.resize(E);
      tcol.resize(E);
    }
    std::printf("abi_host: captured graph, 3 replays on new padded edge lists %s\n",
                cap_ok ? "bit-exact" : "DIFFERS");
    (void)hipGraphExecDestroy(exec);
    (void)hipGraphDestroy(graph);

    // ---- dropout under capture: the mask is keyed by seed + *word ----
    const size_t nf = (size_t)n * F;
    std::vector<float> h(nf), gam(F, 1.25f), bet(F, 0.1f), oa(nf), ob(nf), oc(nf);
    for (auto& v : h) v = ((float)(lcg(seed) % 20001) - 10000.f) / 4096.f;
    float *d_h, *d_gam, *d_bet, *d_o;
    uint64_t* d_word;
    HIP_OK(hipMalloc(&d_h, sizeof(float) * nf));
    HIP_OK(hipMalloc(&d_o, sizeof(float) * nf));
    HIP_OK(hipMalloc(&d_gam, sizeof(float) * F));
    HIP_OK(hipMalloc(&d_bet, sizeof(float) * F));
    HIP_OK(hipMalloc(&d_word, sizeof(uint64_t)));
    HIP_OK(hipMemcpy(d_h, h.data(), sizeof(float) * nf, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_gam, gam.data(), sizeof(float) * F, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_bet, bet.data(), sizeof(float) * F, hipMemcpyHostToDevice));
    auto post = [&](uint64_t sd) {
      return sldm_post_fwd(SLDM_F32, d_h, F, n, F, nullptr, d_gam, d_bet, 1e-5f, 0.1f, 0.25f, sd, 0,
                           SLDM_F32, d_o, nullptr, nullptr, st);
    };
    HIP_OK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    sldm_set_dropout_seed_source(d_word);
    SLDM_CALL(post(7));
    sldm_set_dropout_seed_source(nullptr);
    HIP_OK(hipStreamEndCapture(st, &graph));
    HIP_OK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    const uint64_t words[2] = {100, 200};
    std::vector<float>* outs[2] = {&oa, &ob};
    for (int rep = 0; rep < 2; ++rep) {
      HIP_OK(hipMemcpy(d_word, &words[rep], sizeof(uint64_t), hipMemcpyHostToDevice));
      HIP_OK(hipGraphLaunch(exec, st));
      HIP_OK(hipStreamSynchronize(st));
      HIP_OK(hipMemcpy(outs[rep]->data(), d_o, sizeof(float) * nf, hipMemcpyDeviceToHost));
    }
    SLDM_CALL(post(7 + 200));                      // eager, host seed only
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(oc.data(), d_o, sizeof(float) * nf, hipMemcpyDeviceToHost));
    size_t zeros = 0;
    for (float v : ob) zeros += v == 0.f;
    drop_ok = std::memcmp(ob.data(), oc.data(), sizeof(float) * nf) == 0 &&
              std::memcmp(oa.data(), ob.data(), sizeof(float) * nf) != 0 &&
              zeros > nf / 5 && zeros < nf * 3 / 10;
    std::printf("abi_host: dropout seed word: replay == eager(seed + word) %s, masks of two "
                "words %s, dropped fraction %.3f\n",
                std::memcmp(ob.data(), oc.data(), sizeof(float) * nf) == 0 ? "bit-exact" : "DIFFERS",
                std::memcmp(oa.data(), ob.data(), sizeof(float) * nf) != 0 ? "differ" : "DIFFERS NOT",
                (double)zeros / (double)nf);
    (void)hipGraphExecDestroy(exec);
    (void)hipGraphDestroy(graph);
    for (void* ptr : {(void*)d_h, (void*)d_o, (void*)d_gam, (void*)d_bet, (void*)d_word})
      (void)hipFree(ptr);
  }
  for (void* ptr : {(void*)d_ei, (void*)d_x, (void*)d_add, (void*)d_out, (void*)d_dx,
                    (void*)d_rp, (void*)d_trp, (void*)d_col, (void*)d_tcol, (void*)d_bad, d_ws})
    (void)hipFree(ptr);
  (void)hipStreamDestroy(st);
  return ok && cap_ok && drop_ok ? 0 : 1;
}
