// PyTorch custom operators of the SageBlock hot path: TORCH_LIBRARY(sldm, ...).
//
// The reference calls SageBlock from Python (src/models/grusage.py:182,
// src/models/map/mapencoder.py:37) and PyG dispatches one ATen op per step
// (index_select, scatter_add_, linear, layer_norm, leaky_relu, dropout).
// Here the same steps are dispatcher-visible operators whose CUDA (= HIP on
// ROCm) implementations run the hand-written gfx950 kernels through the C ABI
// of libsldm_sage.so (include/sldm_sage.h) -- one C++ call per layer, or per
// whole stack, and direction, instead of one Python -> C call per kernel:
//
//   sldm::csr_build          edge_index -> CSR by destination (+ transpose)
//   sldm::gather_rows        the CSR row gather (mean aggregation / transpose sum)
//   sldm::mean_aggregate     PyG propagate + MeanAggregation (+ _bwd)
//   sldm::sage_layer         SAGEConv(mean) + LayerNorm + act + dropout (+ _bwd)
//   sldm::sage_stack_fwd/bwd all layers of a SageBlock, fused layer boundaries
//   sldm::segment_pool       global mean / max pooling over batch (+ _bwd)
//   sldm::timing_*           HIP-event brackets around each kernel (bench.py)
//
// Outputs come from the PyTorch caching allocator (at::empty on the input's
// device); every kernel is enqueued on the current HIP stream of that device;
// inputs are borrowed for the call.  Autograd is wired in Python
// (sldm_sage/torch_ops.py: torch.library.register_autograd for the per-op
// forms, one autograd.Function for the stack).  A failed C-ABI call raises a
// c10::Error carrying sldm_last_error().
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <hip/hip_runtime_api.h>

#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "sldm_sage.h"

namespace {

using at::Tensor;
using c10::optional;

// ---------------------------------------------------------------- helpers --
int dtype_code(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return SLDM_F32;
  if (t.scalar_type() == at::kBFloat16) return SLDM_BF16;
  TORCH_CHECK(false, "sldm: unsupported dtype ", t.scalar_type(), " (float32 or bfloat16)");
}

void require_gpu(const Tensor& ref, std::initializer_list<const Tensor*> ts) {
  TORCH_CHECK(ref.is_cuda(), "sldm: tensors must be on a ROCm device (no CPU fallback), got ",
              ref.device());
  for (const Tensor* t : ts)
    if (t && t->defined() && t->numel())
      TORCH_CHECK(t->device() == ref.device(), "sldm: tensors on different devices (",
                  ref.device(), ", ", t->device(), ")");
}

void check(int rc, const char* what) {
  TORCH_CHECK(rc == SLDM_OK, what, " failed (status ", rc, "): ", sldm_last_error());
}

// ROCm builds of PyTorch present HIP devices under the "cuda" device type: the
// guard and the stream query are the masquerading ones.
using DeviceGuard = c10::hip::HIPGuardMasqueradingAsCUDA;
void* stream_of(const Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

const int32_t* i32(const Tensor& t) { return t.numel() ? t.data_ptr<int32_t>() : nullptr; }

// fp32 contiguous view of a small parameter (bias / gamma / beta)
Tensor f32c(const Tensor& t) {
  if (t.scalar_type() == at::kFloat && t.is_contiguous()) return t;
  return t.to(at::kFloat).contiguous();
}
const float* f32p(const optional<Tensor>& t, Tensor& keep) {
  if (!t.has_value() || !t->defined()) return nullptr;
  keep = f32c(*t);
  return keep.data_ptr<float>();
}

// ----------------------------------------------------------------- timing --
// HIP events around each kernel launch, on the launch stream (bench.py's
// per-kernel table and its live roofline figure).  Off by default.
struct TimingRec {
  std::string name;
  hipEvent_t start, stop;
  double units;
  bool failed = false;
};
std::mutex g_tmu;
bool g_timing_on = false;
std::set<std::string> g_timing_names;   // empty: every kernel
std::vector<TimingRec> g_timing_recs;

struct Timed {
  bool on = false;
  TimingRec rec{};
  hipStream_t stream;
  Timed(const char* name, double units, void* stream_) : stream((hipStream_t)stream_) {
    {
      std::lock_guard<std::mutex> lk(g_tmu);
      on = g_timing_on && (g_timing_names.empty() || g_timing_names.count(name));
    }
    if (!on) return;
    rec.name = name;
    rec.units = units;
    TORCH_CHECK(hipEventCreate(&rec.start) == hipSuccess && hipEventCreate(&rec.stop) == hipSuccess,
                "sldm: hipEventCreate failed");
    const hipError_t e = hipEventRecord(rec.start, stream);
    TORCH_CHECK(e == hipSuccess, "sldm: hipEventRecord before ", name, ": ", hipGetErrorString(e));
  }
  ~Timed() {
    if (!on) return;
    rec.failed = hipEventRecord(rec.stop, stream) != hipSuccess;   // reported by timing_take
    std::lock_guard<std::mutex> lk(g_tmu);
    g_timing_recs.push_back(rec);
  }
};

void timing_set(bool on, c10::List<std::string> names) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_timing_on = on;
  g_timing_names.clear();
  for (const std::string& n : names) g_timing_names.insert(n);
}

std::tuple<std::vector<std::string>, std::vector<double>, std::vector<double>> timing_take() {
  std::vector<TimingRec> recs;
  {
    std::lock_guard<std::mutex> lk(g_tmu);
    recs.swap(g_timing_recs);
  }
  std::vector<std::string> names;
  std::vector<double> ms, units;
  hipError_t first_err = hipSuccess;
  std::string first_name;
  for (TimingRec& r : recs) {
    float t = 0.f;
    hipError_t e = r.failed ? hipErrorUnknown : hipEventSynchronize(r.stop);
    if (e == hipSuccess) e = hipEventElapsedTime(&t, r.start, r.stop);
    if (e != hipSuccess && first_err == hipSuccess) {
      first_err = e;
      first_name = r.name;
    }
    (void)hipEventDestroy(r.start);
    (void)hipEventDestroy(r.stop);
    names.push_back(r.name);
    ms.push_back(t);
    units.push_back(r.units);
  }
  TORCH_CHECK(first_err == hipSuccess, "sldm::timing_take: the events around ", first_name,
              " report ", hipGetErrorString(first_err));
  return {names, ms, units};
}

// ------------------------------------------------------------------ graph --
// A graph crosses the op boundary as 12 tensors + 9 ints (SageGraph.packed()):
//   [rowptr, col, t_rowptr, t_col, hub_rows, hub_chunk_ptr, chunk_row, chunk_beg,
//    t_hub_rows, t_hub_chunk_ptr, t_chunk_row, t_chunk_beg]   (absent: 0 elements)
//   [has_transpose, num_hubs, num_chunks, chunk_len, max_deg, t_num_hubs, ...]
struct HubView {
  const int32_t *hub_rows = nullptr, *chunk_ptr = nullptr, *chunk_row = nullptr,
                *chunk_beg = nullptr;
  int64_t num_hubs = 0, num_chunks = 0;
  int32_t chunk_len = 1, max_deg = 0;
  bool on() const { return num_hubs > 0; }
};
struct GraphView {
  Tensor rowptr, col, t_rowptr, t_col;
  bool has_t = false;
  HubView hub, t_hub;
  int64_t edges() const { return col.numel(); }
};

HubView hub_view(const at::TensorList& g, size_t at0, at::IntArrayRef meta, size_t m0) {
  HubView h;
  h.num_hubs = meta[m0];
  h.num_chunks = meta[m0 + 1];
  h.chunk_len = (int32_t)meta[m0 + 2];
  h.max_deg = (int32_t)meta[m0 + 3];
  if (h.num_hubs > 0) {
    h.hub_rows = i32(g[at0]);
    h.chunk_ptr = i32(g[at0 + 1]);
    h.chunk_row = i32(g[at0 + 2]);
    h.chunk_beg = i32(g[at0 + 3]);
    TORCH_CHECK(h.hub_rows && h.chunk_ptr && h.chunk_row && h.chunk_beg && h.num_chunks > 0,
                "sldm: incomplete hub plan");
  }
  return h;
}

GraphView graph_view(const at::TensorList& g, at::IntArrayRef meta) {
  TORCH_CHECK(g.size() == 12 && meta.size() == 9, "sldm: graph must be 12 tensors + 9 ints, got ",
              g.size(), " + ", meta.size());
  GraphView v;
  v.rowptr = g[0];
  v.col = g[1];
  v.t_rowptr = g[2];
  v.t_col = g[3];
  v.has_t = meta[0] != 0;
  for (int i = 0; i < 4; ++i)
    TORCH_CHECK(g[i].scalar_type() == at::kInt && g[i].is_contiguous(),
                "sldm: CSR arrays must be contiguous int32");
  v.hub = hub_view(g, 4, meta, 1);
  v.t_hub = hub_view(g, 8, meta, 5);
  return v;
}

// ----------------------------------------------------------------- gather --
// out[i] = (addend[i] +) sum_{k in row i} x[col[k]] (/ max(1, deg_i) if mean)
Tensor gather(const Tensor& x_in, const Tensor& rowptr, const Tensor& col, const Tensor* order,
              int64_t num_rows, bool mean, const Tensor* addend_in, Tensor out, const HubView& hub,
              const char* name, int64_t edges = -1) {
  Tensor x = (x_in.dim() == 2 && x_in.stride(1) == 1) ? x_in : x_in.contiguous();
  TORCH_CHECK(x.dim() == 2, "sldm::gather_rows: x must be [N, F]");
  const int64_t F = x.size(1);
  if (!out.defined()) out = at::empty({num_rows, F}, x.options());
  Tensor addend;
  if (addend_in && addend_in->defined()) {
    addend = *addend_in;
    if (addend.scalar_type() != out.scalar_type() || addend.stride(-1) != 1)
      addend = addend.to(out.scalar_type()).contiguous();
  }
  if (num_rows == 0 || F == 0) return out;
  const int64_t E = col.numel();
  const int64_t s = x.element_size();
  const double bytes = (double)(edges < 0 ? E : edges) * (4 + F * s) + (num_rows + 1) * 4.0 +
                       (double)num_rows * F * s * (addend.defined() ? 2 : 1);
  const int32_t* colp = E ? i32(col) : i32(rowptr);
  const int32_t* ordp = (order && order->defined() && order->numel()) ? i32(*order) : nullptr;
  void* st = stream_of(x);
  Timed timed(name, bytes, st);
  if (hub.on()) {
    Tensor partials = at::empty({hub.num_chunks, F}, x.options().dtype(at::kFloat));
    check(sldm_gather_rows_split(
              dtype_code(x), x.data_ptr(), x.stride(0), i32(rowptr), colp, ordp, num_rows, F,
              mean ? 1 : 0, addend.defined() ? addend.data_ptr() : nullptr,
              addend.defined() ? addend.stride(0) : 0, dtype_code(out), out.data_ptr(),
              out.stride(0), hub.hub_rows, hub.chunk_ptr, hub.num_hubs, hub.chunk_row,
              hub.chunk_beg, hub.num_chunks, hub.chunk_len, hub.max_deg,
              partials.data_ptr<float>(), st),
          "sldm_gather_rows_split");
    return out;
  }
  check(sldm_gather_rows(dtype_code(x), x.data_ptr(), x.stride(0), i32(rowptr), colp, ordp,
                         num_rows, F, mean ? 1 : 0,
                         addend.defined() ? addend.data_ptr() : nullptr,
                         addend.defined() ? addend.stride(0) : 0, dtype_code(out), out.data_ptr(),
                         out.stride(0), st),
        "sldm_gather_rows");
  return out;
}

// ------------------------------------------------------------ dense pieces --
Tensor weight_cat(const Tensor& wl, const Tensor& wr, at::ScalarType dt) {
  return at::cat({wl, wr}, 1).to(dt).contiguous();
}

struct FwdOut {
  Tensor out, xhat, rstd;
};
// out = dropout(act(LN([agg | x] wcat^T + bias)))
FwdOut dense_fwd(const Tensor& agg, const Tensor& x, const Tensor& wcat,
                 const optional<Tensor>& bias, const Tensor& gamma, const Tensor& beta, double eps,
                 double slope, double drop_p, int64_t seed, bool save, int64_t row_offset) {
  const int64_t n = x.size(0), fi = x.size(1), fo = wcat.size(0);
  TORCH_CHECK(agg.sizes() == x.sizes() && agg.stride(1) == 1 && x.stride(1) == 1 &&
                  wcat.is_contiguous() && wcat.size(1) == 2 * fi && wcat.scalar_type() == x.scalar_type(),
              "sldm::sage_layer: operand layout");
  FwdOut o;
  o.out = at::empty({n, fo}, x.options());
  if (save) {
    o.xhat = at::empty({n, fo}, x.options());
    o.rstd = at::empty({n}, x.options().dtype(at::kFloat));
  }
  Tensor kb, kg = f32c(gamma), kbeta = f32c(beta);
  const float* bp = f32p(bias, kb);
  void* st = stream_of(x);
  Timed timed("dense_fwd", (double)(2 * n * fi + n * fo * (save ? 2 : 1)) * x.element_size(), st);
  check(sldm_sage_dense_fwd(dtype_code(x), agg.data_ptr(), agg.stride(0), fi, x.data_ptr(),
                            x.stride(0), fi, wcat.data_ptr(), n, fo, bp, kg.data_ptr<float>(),
                            kbeta.data_ptr<float>(), (float)eps, (float)slope, (float)drop_p,
                            (uint64_t)seed, row_offset, o.out.data_ptr(),
                            save ? o.xhat.data_ptr() : nullptr,
                            save ? o.rstd.data_ptr<float>() : nullptr, st),
        "sldm_sage_dense_fwd");
  return o;
}

struct PostBwd {
  Tensor dh, dgamma, dbeta, dbias;
};
PostBwd post_bwd(const Tensor& dout_in, const Tensor& xhat, const Tensor& rstd, const Tensor& gamma,
                 const Tensor& beta, double slope, double drop_p, int64_t seed,
                 int64_t row_offset) {
  const int64_t N = xhat.size(0), F = xhat.size(1);
  Tensor dout = dout_in;
  if (dout.scalar_type() != xhat.scalar_type() || dout.stride(1) != 1 || dout.stride(0) != F)
    dout = dout.to(xhat.scalar_type()).contiguous();
  const int np = sldm_post_num_partials(N, F);
  PostBwd r;
  r.dh = at::empty({N, F}, xhat.options());
  Tensor partials = at::empty({np, 3 * F}, xhat.options().dtype(at::kFloat));
  Tensor cols = at::empty({3 * F}, xhat.options().dtype(at::kFloat));
  Tensor kg = f32c(gamma), kb = f32c(beta);
  void* st = stream_of(xhat);
  {
    Timed timed("post_bwd", (double)N * F * 3 * xhat.element_size(), st);
    check(sldm_post_bwd(dtype_code(xhat), dout.data_ptr(), xhat.data_ptr(), nullptr,
                        rstd.data_ptr<float>(), N, F, kg.data_ptr<float>(), kb.data_ptr<float>(),
                        (float)slope, (float)drop_p, (uint64_t)seed, row_offset, dtype_code(xhat),
                        r.dh.data_ptr(), partials.data_ptr<float>(), np, st),
          "sldm_post_bwd");
    check(sldm_colsum(partials.data_ptr<float>(), np, 3 * F, cols.data_ptr<float>(), st),
          "sldm_colsum");
  }
  r.dgamma = cols.slice(0, 0, F);
  r.dbeta = cols.slice(0, F, 2 * F);
  r.dbias = cols.slice(0, 2 * F, 3 * F);
  return r;
}

// Fused layer boundary: transpose gather of layer l (+ addend) straight into
// layer l-1's LayerNorm / act / dropout backward.
PostBwd gather_post_bwd(const Tensor& g, const GraphView& gr, const Tensor& addend,
                        const Tensor& xhat, const Tensor& rstd, const Tensor& gamma,
                        const Tensor& beta, double slope, double drop_p, int64_t seed) {
  const int64_t N = xhat.size(0), F = xhat.size(1);
  TORCH_CHECK(g.scalar_type() == xhat.scalar_type() && addend.scalar_type() == xhat.scalar_type() &&
                  g.stride(1) == 1 && addend.stride(1) == 1 && xhat.is_contiguous() &&
                  g.size(1) == F && addend.size(0) == N && addend.size(1) == F,
              "sldm::sage_stack_bwd: boundary operand layout");
  const int np = sldm_gather_post_bwd_num_partials(N, F);
  PostBwd r;
  r.dh = at::empty({N, F}, xhat.options());
  Tensor partials = at::empty({np, 3 * F}, xhat.options().dtype(at::kFloat));
  Tensor cols = at::empty({3 * F}, xhat.options().dtype(at::kFloat));
  Tensor kg = f32c(gamma), kb = f32c(beta);
  const int64_t E = gr.t_col.numel(), s = xhat.element_size();
  void* st = stream_of(xhat);
  {
    Timed timed("gather_post_bwd",
                (double)E * (4 + F * s) + (N + 1) * 4.0 + 3.0 * N * F * s + 4.0 * N, st);
    check(sldm_gather_post_bwd(dtype_code(xhat), g.data_ptr(), g.stride(0), i32(gr.t_rowptr),
                               E ? i32(gr.t_col) : i32(gr.t_rowptr), nullptr, addend.data_ptr(),
                               addend.stride(0), N, F, xhat.data_ptr(), rstd.data_ptr<float>(),
                               kg.data_ptr<float>(), kb.data_ptr<float>(), (float)slope,
                               (float)drop_p, (uint64_t)seed, 0, r.dh.data_ptr(),
                               partials.data_ptr<float>(), np, st),
          "sldm_gather_post_bwd");
    check(sldm_colsum(partials.data_ptr<float>(), np, 3 * F, cols.data_ptr<float>(), st),
          "sldm_colsum");
  }
  r.dgamma = cols.slice(0, 0, F);
  r.dbeta = cols.slice(0, F, 2 * F);
  r.dbias = cols.slice(0, 2 * F, 3 * F);
  return r;
}

// [dAgg / deg | dx_root] = dh [W_l | W_r] as two contiguous [N, F_in] tensors
std::pair<Tensor, Tensor> bwd_data(const Tensor& dh, const Tensor& wl, const Tensor& wr,
                                   const Tensor& rowptr) {
  const int64_t n = dh.size(0), k = dh.size(1);
  const int64_t fi = wl.size(1);
  // [W_l | W_r]^T = [W_l^T ; W_r^T], [2 F_in, F_out], built by one copy kernel
  Tensor wt = at::cat({wl.t(), wr.t()}, 0).to(dh.scalar_type()).contiguous();
  void* st = stream_of(dh);
  Timed timed("dense_bwd_data", (double)(n * k + n * 2 * fi) * dh.element_size(), st);
  if (fi % 4 == 0) {
    Tensor g = at::empty({n, fi}, dh.options()), dxr = at::empty({n, fi}, dh.options());
    check(sldm_gemm_nt_rowscale(dtype_code(dh), dh.data_ptr(), dh.stride(0), k, wt.data_ptr(),
                                wt.stride(0), n, 2 * fi, i32(rowptr), fi, g.data_ptr(),
                                g.stride(0), dxr.data_ptr(), dxr.stride(0), st),
          "sldm_gemm_nt_rowscale");
    return {g, dxr};
  }
  Tensor buf = at::empty({n, 2 * fi}, dh.options());
  check(sldm_gemm_nt_rowscale(dtype_code(dh), dh.data_ptr(), dh.stride(0), k, wt.data_ptr(),
                              wt.stride(0), n, 2 * fi, i32(rowptr), fi, buf.data_ptr(),
                              buf.stride(0), nullptr, 0, st),
        "sldm_gemm_nt_rowscale");
  return {buf.slice(1, 0, fi), buf.slice(1, fi, 2 * fi)};
}

// (dW_l, dW_r) = (dh^T agg, dh^T x), fp32
std::pair<Tensor, Tensor> bwd_weight(const Tensor& dh, const Tensor& agg, const Tensor& x) {
  const int64_t rows = dh.size(0), mo = dh.size(1), n0 = agg.size(1), n1 = x.size(1);
  TORCH_CHECK(dh.stride(1) == 1 && agg.stride(1) == 1 && x.stride(1) == 1,
              "sldm::sage_layer_bwd: operand layout");
  const size_t ws_bytes = sldm_gemm_tn_workspace_bytes(rows, mo, n0 + n1);
  Tensor ws = at::empty({(int64_t)ws_bytes}, dh.options().dtype(at::kByte));
  Tensor o0 = at::empty({mo, n0}, dh.options().dtype(at::kFloat));
  Tensor o1 = at::empty({mo, n1}, dh.options().dtype(at::kFloat));
  void* st = stream_of(dh);
  Timed timed("dense_bwd_weight", (double)rows * (mo + n0 + n1) * dh.element_size(), st);
  check(sldm_gemm_tn_split(dtype_code(dh), dh.data_ptr(), dh.stride(0), mo, agg.data_ptr(),
                           agg.stride(0), n0, x.data_ptr(), x.stride(0), n1, rows,
                           o0.data_ptr<float>(), o1.data_ptr<float>(), ws.data_ptr(), ws_bytes, st),
        "sldm_gemm_tn_split");
  return {o0, o1};
}

Tensor as_dtype(const Tensor& t, const Tensor& like) {
  return t.scalar_type() == like.scalar_type() ? t : t.to(like.scalar_type());
}

Tensor prep_x(const Tensor& x) {
  TORCH_CHECK(x.dim() == 2, "sldm: x must be [N, F], got ", x.sizes());
  Tensor r = x;
  if (r.scalar_type() != at::kFloat && r.scalar_type() != at::kBFloat16) r = r.to(at::kFloat);
  return r.contiguous();
}

// ---------------------------------------------------------------- the ops --
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> op_csr_build(const Tensor& edge_index,
                                                                 int64_t num_nodes, bool transpose) {
  require_gpu(edge_index, {});
  DeviceGuard guard(edge_index.device());
  TORCH_CHECK(edge_index.dim() == 2 && edge_index.size(0) == 2, "edge_index must be [2, E], got ",
              edge_index.sizes());
  TORCH_CHECK(edge_index.scalar_type() == at::kLong || edge_index.scalar_type() == at::kInt,
              "edge_index must be int64 or int32, got ", edge_index.scalar_type());
  Tensor ei = edge_index.contiguous();
  const int64_t E = ei.size(1), N = num_nodes;
  auto io = ei.options().dtype(at::kInt);
  Tensor rowptr = at::empty({N + 1}, io), col = at::empty({E}, io);
  Tensor t_rowptr = at::empty({transpose ? N + 1 : 0}, io);
  Tensor t_col = at::empty({transpose ? E : 0}, io);
  Tensor bad = at::zeros({1}, io);
  const size_t wsb = sldm_csr_workspace_bytes(E, N);
  Tensor ws = at::empty({(int64_t)wsb}, ei.options().dtype(at::kByte));
  Tensor dummy = at::empty({1}, io);                       // a valid pointer for E == 0
  void* st = stream_of(ei);
  Timed timed("csr_build", (double)E, st);
  check(sldm_csr_build(ei.data_ptr(), ei.scalar_type() == at::kLong, E, N,
                       rowptr.data_ptr<int32_t>(), E ? col.data_ptr<int32_t>() : dummy.data_ptr<int32_t>(),
                       transpose ? t_rowptr.data_ptr<int32_t>() : nullptr,
                       transpose ? (E ? t_col.data_ptr<int32_t>() : dummy.data_ptr<int32_t>()) : nullptr,
                       bad.data_ptr<int32_t>(), ws.data_ptr(), wsb, st),
        "sldm_csr_build");
  return {rowptr, col, t_rowptr, t_col, bad};
}

Tensor op_gather_rows(const Tensor& x, const Tensor& rowptr, const Tensor& col, int64_t num_rows,
                      bool mean, const optional<Tensor>& addend, const optional<Tensor>& order,
                      at::TensorList hub, at::IntArrayRef hub_meta, std::string name,
                      int64_t edges) {
  require_gpu(x, {&rowptr, &col});
  DeviceGuard guard(x.device());
  HubView hv;
  if (!hub.empty()) {
    TORCH_CHECK(hub.size() == 4 && hub_meta.size() == 4, "sldm::gather_rows: hub plan is 4 tensors + 4 ints");
    hv = hub_view(hub, 0, hub_meta, 0);
  }
  return gather(x, rowptr, col, order.has_value() ? &*order : nullptr, num_rows, mean,
                addend.has_value() ? &*addend : nullptr, Tensor(), hv, name.c_str(), edges);
}

Tensor op_mean_aggregate(const Tensor& x_in, at::TensorList graph, at::IntArrayRef meta) {
  require_gpu(x_in, {});
  DeviceGuard guard(x_in.device());
  GraphView g = graph_view(graph, meta);
  Tensor x = prep_x(x_in);
  return gather(x, g.rowptr, g.col, nullptr, x.size(0), true, nullptr, Tensor(), g.hub,
                "gather_fwd");
}

Tensor op_mean_aggregate_bwd(const Tensor& grad, at::TensorList graph, at::IntArrayRef meta) {
  require_gpu(grad, {});
  DeviceGuard guard(grad.device());
  GraphView g = graph_view(graph, meta);
  TORCH_CHECK(g.has_t, "SageGraph was built without its transpose; rebuild with transpose=True "
                       "for backward");
  Tensor d = grad.contiguous().clone();
  check(sldm_scale_rows_by_inv_deg(dtype_code(d), d.data_ptr(), d.stride(0), i32(g.rowptr),
                                   d.size(0), d.size(1), stream_of(d)),
        "sldm_scale_rows_by_inv_deg");
  return gather(d, g.t_rowptr, g.t_col, nullptr, d.size(0), false, nullptr, Tensor(), g.t_hub,
                "gather_bwd");
}

// One layer: returns (out, agg, xhat, rstd); xhat / rstd have 0 elements when
// save is false.
std::tuple<Tensor, Tensor, Tensor, Tensor> op_sage_layer(
    const Tensor& x_in, at::TensorList graph, at::IntArrayRef meta, const Tensor& wl,
    const optional<Tensor>& bl, const Tensor& wr, const Tensor& gamma, const Tensor& beta,
    double slope, double drop_p, int64_t seed, double eps, bool save) {
  require_gpu(x_in, {&wl, &wr, &gamma, &beta});
  DeviceGuard guard(x_in.device());
  GraphView g = graph_view(graph, meta);
  Tensor x = prep_x(x_in);
  Tensor agg = gather(x, g.rowptr, g.col, nullptr, x.size(0), true, nullptr, Tensor(), g.hub,
                      "gather_fwd");
  Tensor wcat = weight_cat(wl, wr, x.scalar_type());
  FwdOut o = dense_fwd(agg, x, wcat, bl, gamma, beta, eps, slope, drop_p, seed, save, 0);
  if (!save) {
    o.xhat = at::empty({0}, x.options());
    o.rstd = at::empty({0}, x.options().dtype(at::kFloat));
  }
  return {o.out, agg, o.xhat, o.rstd};
}

// Backward of sage_layer: (dx, dW_l, db_l, dW_r, dgamma, dbeta); dx has 0
// elements when need_dx is false.
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> op_sage_layer_bwd(
    const Tensor& dout, const Tensor& x, const Tensor& agg, const Tensor& xhat, const Tensor& rstd,
    at::TensorList graph, at::IntArrayRef meta, const Tensor& wl, const Tensor& wr,
    const Tensor& gamma, const Tensor& beta, double slope, double drop_p, int64_t seed,
    bool need_dx) {
  require_gpu(x, {&dout, &wl, &wr});
  DeviceGuard guard(x.device());
  GraphView g = graph_view(graph, meta);
  PostBwd pb = post_bwd(dout, xhat, rstd, gamma, beta, slope, drop_p, seed, 0);
  auto [dwl, dwr] = bwd_weight(pb.dh, agg, x);
  Tensor dx = at::empty({0}, x.options());
  if (need_dx) {
    TORCH_CHECK(g.has_t, "SageGraph was built without its transpose; rebuild with transpose=True "
                         "for backward");
    auto [gd, dxr] = bwd_data(pb.dh, wl, wr, g.rowptr);
    dx = gather(gd, g.t_rowptr, g.t_col, nullptr, x.size(0), false, &dxr, Tensor(), g.t_hub,
                "gather_bwd");
  }
  return {dx, as_dtype(dwl, wl), as_dtype(pb.dbias, wl), as_dtype(dwr, wr),
          as_dtype(pb.dgamma, gamma), as_dtype(pb.dbeta, beta)};
}

// All layers forward.  params: 5 per layer (W_l, b_l, W_r, gamma, beta).
// Returns [out, then per layer: agg, xhat, rstd, (layer input for l > 0)]:
//   saved[4 l + 0] = input of layer l (x for l = 0: returned as given, prepared)
//   saved[4 l + 1] = agg, [4 l + 2] = xhat, [4 l + 3] = rstd
// as a flat list: [out, saved...].
std::vector<Tensor> op_sage_stack_fwd(const Tensor& x_in, at::TensorList graph,
                                      at::IntArrayRef meta, at::TensorList params,
                                      at::ArrayRef<double> slopes, at::ArrayRef<double> drops,
                                      at::IntArrayRef seeds, at::ArrayRef<double> eps, bool save) {
  require_gpu(x_in, {});
  DeviceGuard guard(x_in.device());
  GraphView g = graph_view(graph, meta);
  const size_t L = slopes.size();
  TORCH_CHECK(params.size() == 5 * L && drops.size() == L && seeds.size() == L && eps.size() == L,
              "sldm::sage_stack_fwd: 5 parameters and 4 scalars per layer");
  Tensor h = prep_x(x_in);
  std::vector<Tensor> res(1);
  for (size_t l = 0; l < L; ++l) {
    const Tensor &wl = params[5 * l], &bl = params[5 * l + 1], &wr = params[5 * l + 2],
                 &gamma = params[5 * l + 3], &beta = params[5 * l + 4];
    Tensor agg = gather(h, g.rowptr, g.col, nullptr, h.size(0), true, nullptr, Tensor(), g.hub,
                        "gather_fwd");
    Tensor wcat = weight_cat(wl, wr, h.scalar_type());
    FwdOut o = dense_fwd(agg, h, wcat, bl, gamma, beta, eps[l], slopes[l], drops[l], seeds[l],
                         save, 0);
    if (save) {
      res.push_back(h);
      res.push_back(agg);
      res.push_back(o.xhat);
      res.push_back(o.rstd);
    }
    h = o.out;
  }
  res[0] = h;
  return res;
}

// All layers backward, layer boundaries fused (the transpose gather of layer
// l and the post backward of layer l-1 in one kernel) unless the transpose
// graph has high-degree rows.  Returns [dx (0 elements if !need_dx), then 5
// gradients per layer in parameter order].
std::vector<Tensor> op_sage_stack_bwd(const Tensor& dout, at::TensorList saved,
                                      at::TensorList graph, at::IntArrayRef meta,
                                      at::TensorList params, at::ArrayRef<double> slopes,
                                      at::ArrayRef<double> drops, at::IntArrayRef seeds,
                                      bool need_dx, bool fuse) {
  require_gpu(dout, {});
  DeviceGuard guard(dout.device());
  GraphView g = graph_view(graph, meta);
  const int64_t L = (int64_t)slopes.size();
  TORCH_CHECK((int64_t)params.size() == 5 * L && (int64_t)saved.size() == 4 * L && L > 0,
              "sldm::sage_stack_bwd: 5 parameters and 4 saved tensors per layer");
  TORCH_CHECK(g.has_t || (L == 1 && !need_dx),
              "SageGraph was built without its transpose; rebuild with transpose=True for backward");
  const Tensor& x_in = saved[0];
  std::vector<Tensor> grads(1 + 5 * L);
  grads[0] = at::empty({0}, x_in.options());
  const int64_t top = L - 1;
  PostBwd pb = post_bwd(dout, saved[4 * top + 2], saved[4 * top + 3], params[5 * top + 3],
                        params[5 * top + 4], slopes[top], drops[top], seeds[top], 0);
  for (int64_t i = top; i >= 0; --i) {
    const Tensor &h = saved[4 * i], &agg = saved[4 * i + 1];
    const Tensor &wl = params[5 * i], &wr = params[5 * i + 2], &gamma = params[5 * i + 3],
                 &beta = params[5 * i + 4];
    auto [dwl, dwr] = bwd_weight(pb.dh, agg, h);
    grads[1 + 5 * i + 0] = as_dtype(dwl, wl);
    grads[1 + 5 * i + 1] = as_dtype(pb.dbias, wl);
    grads[1 + 5 * i + 2] = as_dtype(dwr, wr);
    grads[1 + 5 * i + 3] = as_dtype(pb.dgamma, gamma);
    grads[1 + 5 * i + 4] = as_dtype(pb.dbeta, beta);
    if (i == 0 && !need_dx) break;
    auto [gd, dxr] = bwd_data(pb.dh, wl, wr, g.rowptr);
    if (i == 0) {
      grads[0] = gather(gd, g.t_rowptr, g.t_col, nullptr, h.size(0), false, &dxr, Tensor(),
                        g.t_hub, "gather_bwd");
      break;
    }
    const Tensor &xhat_b = saved[4 * (i - 1) + 2], &rstd_b = saved[4 * (i - 1) + 3];
    const Tensor &gamma_b = params[5 * (i - 1) + 3], &beta_b = params[5 * (i - 1) + 4];
    if (g.t_hub.on() || !fuse) {
      // out-degree hubs: the split transpose gather, then the post backward
      // (the fused kernel sums each row in one row group)
      Tensor dxi = gather(gd, g.t_rowptr, g.t_col, nullptr, h.size(0), false, &dxr, Tensor(),
                          g.t_hub, "gather_bwd");
      pb = post_bwd(dxi, xhat_b, rstd_b, gamma_b, beta_b, slopes[i - 1], drops[i - 1],
                    seeds[i - 1], 0);
    } else {
      pb = gather_post_bwd(gd, g, dxr, xhat_b, rstd_b, gamma_b, beta_b, slopes[i - 1],
                           drops[i - 1], seeds[i - 1]);
    }
  }
  return grads;
}

// ------------------------------------------------------------------ pooling --
// mode bit 1: mean, bit 2: max.  Returns (out [B, F or 2F], max_divisor,
// max_first_row); the last two have 0 elements when unused.
std::tuple<Tensor, Tensor, Tensor> op_segment_pool(const Tensor& x_in, const Tensor& seg_rowptr,
                                                   const Tensor& member, const Tensor& piece_ptr,
                                                   int64_t num_segments, int64_t num_pieces,
                                                   int64_t mode, bool first_arg) {
  require_gpu(x_in, {&seg_rowptr, &member, &piece_ptr});
  DeviceGuard guard(x_in.device());
  Tensor x = x_in.contiguous();
  const int64_t B = num_segments, F = x.size(1);
  const bool mean = mode & 1, mx = mode & 2;
  Tensor out = at::empty({B, F * ((mean && mx) ? 2 : 1)}, x.options());
  Tensor meanv = mean ? out.slice(1, 0, F) : Tensor();
  Tensor maxv = mx ? out.slice(1, mean ? F : 0, mean ? 2 * F : F) : Tensor();
  Tensor div = at::empty({(mx && !first_arg) ? B : 0, F}, x.options().dtype(at::kFloat));
  Tensor arg = at::empty({(mx && first_arg) ? B : 0, F}, x.options().dtype(at::kInt));
  const size_t wsb = sldm_segment_pool_workspace_bytes(num_pieces, F);
  Tensor ws = at::empty({(int64_t)wsb}, x.options().dtype(at::kByte));
  void* st = stream_of(x);
  Timed timed("pool_fwd", (double)x.numel() * x.element_size(), st);
  check(sldm_segment_pool(dtype_code(x), x.data_ptr(), x.stride(0), i32(seg_rowptr), i32(member),
                          B, i32(piece_ptr), num_pieces, F, mean ? meanv.data_ptr() : nullptr,
                          mean ? meanv.stride(0) : 0, mx ? maxv.data_ptr() : nullptr,
                          mx ? maxv.stride(0) : 0, div.numel() ? div.data_ptr<float>() : nullptr,
                          arg.numel() ? arg.data_ptr<int32_t>() : nullptr, ws.data_ptr(), wsb, st),
        "sldm_segment_pool");
  return {out, div, arg};
}

Tensor op_segment_pool_bwd(const Tensor& gout, const Tensor& x, const Tensor& pooled,
                           const Tensor& div, const Tensor& arg, const Tensor& seg_of,
                           const Tensor& seg_rowptr, int64_t mode) {
  require_gpu(x, {&gout, &seg_of, &seg_rowptr});
  DeviceGuard guard(x.device());
  const int64_t n = x.size(0), F = x.size(1);
  const bool mean = mode & 1, mx = mode & 2;
  Tensor g = gout.to(x.scalar_type());
  if (g.stride(-1) != 1) g = g.contiguous();
  Tensor dmean = mean ? g.slice(1, 0, F) : Tensor();
  Tensor dmax = mx ? g.slice(1, mean ? F : 0, mean ? 2 * F : F) : Tensor();
  Tensor maxv = mx ? pooled.slice(1, mean ? F : 0, mean ? 2 * F : F) : Tensor();
  Tensor dx = at::empty_like(x);
  void* st = stream_of(x);
  Timed timed("pool_bwd", 2.0 * x.numel() * x.element_size(), st);
  check(sldm_segment_pool_bwd(dtype_code(x), x.data_ptr(), x.stride(0),
                              seg_of.data_ptr<int64_t>(), i32(seg_rowptr), n, F,
                              mean ? dmean.data_ptr() : nullptr, mean ? dmean.stride(0) : 0,
                              mx ? maxv.data_ptr() : nullptr, mx ? maxv.stride(0) : 0,
                              mx ? dmax.data_ptr() : nullptr, mx ? dmax.stride(0) : 0,
                              div.numel() ? div.data_ptr<float>() : nullptr,
                              arg.numel() ? arg.data_ptr<int32_t>() : nullptr, dx.data_ptr(),
                              dx.stride(0), st),
        "sldm_segment_pool_bwd");
  return dx;
}

int64_t op_abi_version() { return sldm_abi_version(); }

}  // namespace

TORCH_LIBRARY(sldm, m) {
  m.def("abi_version() -> int", op_abi_version);
  m.def("timing_set(bool on, str[] names) -> ()", timing_set);
  m.def("timing_take() -> (str[], float[], float[])", timing_take);
  m.def("csr_build(Tensor edge_index, int num_nodes, bool transpose) -> "
        "(Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("gather_rows(Tensor x, Tensor rowptr, Tensor col, int num_rows, bool mean, "
        "Tensor? addend, Tensor? order, Tensor[] hub, int[] hub_meta, str name, int edges) -> "
        "Tensor");
  m.def("mean_aggregate(Tensor x, Tensor[] graph, int[] graph_meta) -> Tensor");
  m.def("mean_aggregate_bwd(Tensor grad, Tensor[] graph, int[] graph_meta) -> Tensor");
  m.def("sage_layer(Tensor x, Tensor[] graph, int[] graph_meta, Tensor wl, Tensor? bl, Tensor wr, "
        "Tensor gamma, Tensor beta, float slope, float drop_p, int seed, float eps, bool save) -> "
        "(Tensor, Tensor, Tensor, Tensor)");
  m.def("sage_layer_bwd(Tensor dout, Tensor x, Tensor agg, Tensor xhat, Tensor rstd, "
        "Tensor[] graph, int[] graph_meta, Tensor wl, Tensor wr, Tensor gamma, Tensor beta, "
        "float slope, float drop_p, int seed, bool need_dx) -> "
        "(Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("sage_stack_fwd(Tensor x, Tensor[] graph, int[] graph_meta, Tensor[] params, "
        "float[] slopes, float[] drops, int[] seeds, float[] eps, bool save) -> Tensor[]");
  m.def("sage_stack_bwd(Tensor dout, Tensor[] saved, Tensor[] graph, int[] graph_meta, "
        "Tensor[] params, float[] slopes, float[] drops, int[] seeds, bool need_dx, bool fuse) -> "
        "Tensor[]");
  m.def("segment_pool(Tensor x, Tensor seg_rowptr, Tensor member, Tensor piece_ptr, "
        "int num_segments, int num_pieces, int mode, bool first_arg) -> (Tensor, Tensor, Tensor)");
  m.def("segment_pool_bwd(Tensor gout, Tensor x, Tensor pooled, Tensor div, Tensor arg, "
        "Tensor seg_of, Tensor seg_rowptr, int mode) -> Tensor");
}

TORCH_LIBRARY_IMPL(sldm, CUDA, m) {
  m.impl("csr_build", op_csr_build);
  m.impl("gather_rows", op_gather_rows);
  m.impl("mean_aggregate", op_mean_aggregate);
  m.impl("mean_aggregate_bwd", op_mean_aggregate_bwd);
  m.impl("sage_layer", op_sage_layer);
  m.impl("sage_layer_bwd", op_sage_layer_bwd);
  m.impl("sage_stack_fwd", op_sage_stack_fwd);
  m.impl("sage_stack_bwd", op_sage_stack_bwd);
  m.impl("segment_pool", op_segment_pool);
  m.impl("segment_pool_bwd", op_segment_pool_bwd);
}
