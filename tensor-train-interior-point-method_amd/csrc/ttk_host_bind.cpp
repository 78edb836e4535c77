// Host-side argument packing for the hot einsum / element-wise entry points of libttk.
//
// The TT-IPM host loop issues ~10^5 contraction and copy calls per solve; packing pointers,
// shapes and strides of torch tensors in Python costs ~8 us per call (attribute lookups + a
// ctypes array), more than the kernel itself.  This module reads them natively and calls the
// same C ABI (`include/ttk.h`: ttk_einsum, ttk_copy_nd, ttk_mul_nd) through function pointers
// handed over from the ctypes handle, so both paths share one libttk instance (plan cache,
// event counters).  No device arithmetic happens here; ttk_host_eig.inc adds the step-size
// eigen-ALS's orchestration (host decisions and NumPy's Gaussian stream restated, same libttk calls).
#include <torch/extension.h>

#include <pybind11/numpy.h>

#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <unordered_map>
#include <tuple>
#include <vector>

namespace {

using einsum_fn = int (*)(void *, const char *, const int64_t *, double *, double, double);
using copy_fn = int (*)(void *, const double *, double *, int, const int64_t *, const int64_t *, const int64_t *,
                        double, double);
using mul_fn = int (*)(void *, const double *, const double *, double *, int, const int64_t *, const int64_t *,
                       const int64_t *, const int64_t *, double, double);

using axpby_fn = int (*)(void *, const double *, const double *, double *, int, const int64_t *, const int64_t *,
                         const int64_t *, const int64_t *, double, double, double);
using normalize_fn = int (*)(void *, const double *, double *, int, const int64_t *, const int64_t *);
using scale_ss_fn = int (*)(void *, const double *, double *, int, const int64_t *, const int64_t *, const int64_t *,
                            int, const double *, int);
using dot_dev_fn = int (*)(void *, const double *, const double *, int, const int64_t *, const int64_t *,
                           const int64_t *, double *);
using fill_fn = int (*)(void *, double *, int64_t, double);

einsum_fn g_einsum = nullptr;
axpby_fn g_axpby = nullptr;
normalize_fn g_normalize = nullptr;
scale_ss_fn g_scale_ss = nullptr;
dot_dev_fn g_dot_dev = nullptr;
fill_fn g_fill = nullptr;
copy_fn g_copy = nullptr;
mul_fn g_mul = nullptr;
// one launch stream per host thread: a process may drive several solves at once, one per thread,
// each on its own stream and libttk context (bind() is called once on each such thread)
thread_local void *g_stream = nullptr;
bool g_release_gil = true;

void bind(int64_t einsum_addr, int64_t copy_addr, int64_t mul_addr, int64_t stream) {
  g_einsum = reinterpret_cast<einsum_fn>(einsum_addr);
  g_copy = reinterpret_cast<copy_fn>(copy_addr);
  g_mul = reinterpret_cast<mul_fn>(mul_addr);
  g_stream = reinterpret_cast<void *>(stream);
}

// the element-wise / reduction entry points of dev.py's hot wrappers (same libttk calls as its ctypes
// path; one pybind call instead of ctypes argument packing)
void bind2(int64_t axpby_addr, int64_t normalize_addr, int64_t scale_ss_addr, int64_t dot_dev_addr,
           int64_t fill_addr) {
  g_axpby = reinterpret_cast<axpby_fn>(axpby_addr);
  g_normalize = reinterpret_cast<normalize_fn>(normalize_addr);
  g_scale_ss = reinterpret_cast<scale_ss_fn>(scale_ss_addr);
  g_dot_dev = reinterpret_cast<dot_dev_fn>(dot_dev_addr);
  g_fill = reinterpret_cast<fill_fn>(fill_addr);
}

// output index string -> positions (operand, axis) of each output letter, per (equation)
struct OutMap {
  std::vector<std::pair<int, int>> src;
};
std::unordered_map<std::string, OutMap> g_out;
std::mutex g_out_mu;  // the native eigen-ALS calls this without the GIL, from several solve threads

const OutMap &out_map(const std::string &eq) {
  std::lock_guard<std::mutex> lock(g_out_mu);  // map nodes are stable: the reference outlives the lock
  auto it = g_out.find(eq);
  if (it != g_out.end()) return it->second;
  OutMap m;
  const auto arrow = eq.find("->");
  TORCH_CHECK(arrow != std::string::npos, "einsum: missing '->' in ", eq);
  const std::string lhs = eq.substr(0, arrow), rhs = eq.substr(arrow + 2);
  std::vector<std::string> ins;
  size_t s = 0;
  for (size_t i = 0; i <= lhs.size(); ++i)
    if (i == lhs.size() || lhs[i] == ',') {
      ins.push_back(lhs.substr(s, i - s));
      s = i + 1;
    }
  for (char c : rhs) {
    bool found = false;
    for (int o = 0; o < (int)ins.size() && !found; ++o) {
      const auto p = ins[o].find(c);
      if (p != std::string::npos) {
        m.src.emplace_back(o, (int)p);
        found = true;
      }
    }
    TORCH_CHECK(found, "einsum: output index ", c, " not in inputs of ", eq);
  }
  return g_out.emplace(eq, std::move(m)).first->second;
}

void check(int rc, const char *what) { TORCH_CHECK(rc == 0, "libttk ", what, " failed with status ", rc); }

// out = alpha * einsum(eq, ops) + beta * out (out allocated when None); flags: 256 = fused opt-in.
// release: drop the GIL around the launch (the caller holds it)
at::Tensor einsum_impl(const std::string &eq, const std::vector<at::Tensor> &ops, c10::optional<at::Tensor> out,
                       double alpha, double beta, int64_t flags, bool release) {
  TORCH_CHECK(g_einsum, "ttk_host_bind: bind() not called");
  const int nops = (int)ops.size();
  TORCH_CHECK(nops >= 1 && nops <= 8, "einsum: ", nops, " operands");
  int64_t desc[8 * 34 + 20];
  int64_t pos = 0;
  desc[pos++] = nops | flags;
  for (const auto &o : ops) {
    const int nd = (int)o.dim();
    TORCH_CHECK(nd <= 16, "einsum: operand rank ", nd);
    TORCH_CHECK(o.scalar_type() == at::kDouble && o.device() == ops[0].device(),
                "einsum: operands must be float64 on one device (", eq, ")");
    desc[pos++] = reinterpret_cast<int64_t>(o.data_ptr());
    desc[pos++] = nd;
    const auto sz = o.sizes();
    const auto st = o.strides();
    for (int i = 0; i < nd; ++i) desc[pos++] = sz[i];
    for (int i = 0; i < nd; ++i) desc[pos++] = st[i];
  }
  at::Tensor res;
  if (out.has_value()) {
    res = *out;
    const int nd = (int)res.dim();
    TORCH_CHECK(res.scalar_type() == at::kDouble && res.device() == ops[0].device(), "einsum: out dtype/device");
    const OutMap &m = out_map(eq);
    TORCH_CHECK((size_t)nd == m.src.size(), "einsum: out rank ", nd, " for ", eq);
    for (int i = 0; i < nd; ++i)
      TORCH_CHECK(res.size(i) == ops[m.src[i].first].size(m.src[i].second), "einsum: out shape ", res.sizes(),
                  " does not match ", eq);
    desc[pos++] = 1;
    desc[pos++] = nd;
    const auto st = res.strides();
    for (int i = 0; i < nd; ++i) desc[pos++] = st[i];
  } else {
    const OutMap &m = out_map(eq);
    std::vector<int64_t> shp(m.src.size());
    for (size_t i = 0; i < m.src.size(); ++i) shp[i] = ops[m.src[i].first].size(m.src[i].second);
    res = at::empty(shp, ops[0].options());
    beta = 0.0;
    desc[pos++] = 0;
  }
  double *rp = res.data_ptr<double>();
  int rc;
  if (release) {  // the launch itself touches no Python object: other solve threads may run meanwhile
    pybind11::gil_scoped_release nogil;
    rc = g_einsum(g_stream, eq.c_str(), desc, rp, alpha, beta);
  } else {  // TTK_HOLD_GIL: threads switch only where one waits for the device (dev.py)
    rc = g_einsum(g_stream, eq.c_str(), desc, rp, alpha, beta);
  }
  check(rc, "einsum");
  return res;
}

at::Tensor einsum(const std::string &eq, const std::vector<at::Tensor> &ops, c10::optional<at::Tensor> out,
                  double alpha, double beta, int64_t flags) {
  return einsum_impl(eq, ops, out, alpha, beta, flags, g_release_gil);
}

// A run of einsums over block columns (the block local products of tt_als.py): item = (equation
// index, operands, x column or -1, out column); operand list + x.select(1, xcol) -> out.select(1,
// ocol), accumulated with (alpha, beta), in item order -- the same libttk calls, in the same order,
// as one dev.einsum per item, without a Python slice and wrapper per block.
void einsum_cols(const std::vector<std::string> &eqs,
                 const std::vector<std::tuple<int64_t, std::vector<at::Tensor>, int64_t, int64_t>> &items,
                 const at::Tensor &x, const at::Tensor &out, double alpha, double beta, int64_t flags) {
  for (const auto &it : items) {
    std::vector<at::Tensor> ops = std::get<1>(it);
    const int64_t xc = std::get<2>(it), oc = std::get<3>(it);
    if (xc >= 0) ops.push_back(x.select(1, xc));
    einsum(eqs.at((size_t)std::get<0>(it)), ops, out.select(1, oc), alpha, beta, flags);
  }
}

at::Tensor copy_(at::Tensor dst, const at::Tensor &src, double alpha, double beta) {
  TORCH_CHECK(dst.sizes() == src.sizes(), "copy_: shape mismatch ", dst.sizes(), " vs ", src.sizes());
  int nd = (int)dst.dim();
  int64_t shp[16], ss[16], ds[16];
  TORCH_CHECK(nd <= 16, "copy_: rank ", nd);
  if (nd == 0) {
    nd = 1;
    shp[0] = 1;
    ss[0] = ds[0] = 1;
  } else {
    for (int i = 0; i < nd; ++i) {
      shp[i] = dst.size(i);
      ss[i] = src.stride(i);
      ds[i] = dst.stride(i);
    }
  }
  check(g_copy(g_stream, src.data_ptr<double>(), dst.data_ptr<double>(), nd, shp, ss, ds, alpha, beta), "copy_nd");
  return dst;
}

at::Tensor mul_(at::Tensor dst, const at::Tensor &a, const at::Tensor &b, double alpha, double beta) {
  const int nd = (int)dst.dim();
  TORCH_CHECK(nd >= 1 && nd <= 16 && a.dim() == nd && b.dim() == nd, "mul_: rank mismatch");
  TORCH_CHECK(a.sizes() == dst.sizes() && b.sizes() == dst.sizes(), "mul_: shape mismatch ", a.sizes(), " ",
              b.sizes(), " -> ", dst.sizes());
  int64_t shp[16], as[16], bs[16], ds[16];
  for (int i = 0; i < nd; ++i) {
    shp[i] = dst.size(i);
    as[i] = a.stride(i);
    bs[i] = b.stride(i);
    ds[i] = dst.stride(i);
  }
  check(g_mul(g_stream, a.data_ptr<double>(), b.data_ptr<double>(), dst.data_ptr<double>(), nd, shp, as, bs, ds,
              alpha, beta),
        "mul_nd");
  return dst;
}

int geometry(const at::Tensor &t, int64_t *shp, int64_t *st) {
  const int nd = (int)t.dim();
  TORCH_CHECK(nd <= 16, "rank ", nd);
  for (int i = 0; i < nd; ++i) {
    shp[i] = t.size(i);
    st[i] = t.stride(i);
  }
  return nd;
}

// out = alpha * src + beta * (gamma * src2) (dev.axpby)
at::Tensor axpby(const at::Tensor &src, const at::Tensor &src2, double alpha, double beta, double gamma,
                 c10::optional<at::Tensor> out_opt) {
  at::Tensor out = out_opt.has_value() ? *out_opt : at::empty(src.sizes(), src.options());
  int64_t shp[16], s1[16], s2[16], so[16];
  const int nd = geometry(src, shp, s1);
  TORCH_CHECK(src2.dim() == nd && out.dim() == nd, "axpby: rank mismatch");
  for (int i = 0; i < nd; ++i) {
    s2[i] = src2.stride(i);
    so[i] = out.stride(i);
  }
  check(g_axpby(g_stream, src.data_ptr<double>(), src2.data_ptr<double>(), out.data_ptr<double>(), nd, shp, s1, s2,
                so, alpha, beta, gamma),
        "axpby_nd");
  return out;
}

// src / ||src|| into a new contiguous tensor (dev.normalized)
at::Tensor normalized(const at::Tensor &src) {
  at::Tensor out = at::empty(src.sizes(), src.options());
  int64_t shp[16], st[16];
  int nd = geometry(src, shp, st);
  if (nd == 0) {
    nd = 1;
    shp[0] = st[0] = 1;
  }
  check(g_normalize(g_stream, src.data_ptr<double>(), out.data_ptr<double>(), nd, shp, st), "normalize");
  return out;
}

// src * f(ss[i_axis]) (dev.scale_axis_ss)
at::Tensor scale_axis_ss(const at::Tensor &src, int64_t axis, const at::Tensor &ss, bool invert,
                         c10::optional<at::Tensor> out_opt) {
  at::Tensor out = out_opt.has_value() ? *out_opt : at::empty(src.sizes(), src.options());
  int64_t shp[16], s1[16], so[16];
  const int nd = geometry(src, shp, s1);
  TORCH_CHECK(out.dim() == nd, "scale_axis_ss: rank mismatch");
  for (int i = 0; i < nd; ++i) so[i] = out.stride(i);
  check(g_scale_ss(g_stream, src.data_ptr<double>(), out.data_ptr<double>(), nd, shp, s1, so, (int)axis,
                   ss.data_ptr<double>(), invert ? 1 : 0),
        "scale_axis_ss");
  return out;
}

// sum(x * y) into the device scalar `out` (dev.dot_into)
void dot_into(const at::Tensor &x, const at::Tensor &y, at::Tensor out) {
  TORCH_CHECK(x.sizes() == y.sizes(), "dot_into: shape mismatch ", x.sizes(), " vs ", y.sizes());
  int64_t shp[16], xs[16], ys[16];
  int nd = geometry(x, shp, xs);
  for (int i = 0; i < nd; ++i) ys[i] = y.stride(i);
  if (nd == 0) {
    nd = 1;
    shp[0] = xs[0] = ys[0] = 1;
  }
  check(g_dot_dev(g_stream, x.data_ptr<double>(), y.data_ptr<double>(), nd, shp, xs, ys, out.data_ptr<double>()),
        "dot_nd_dev");
}

// a zero-filled tensor: at::empty + libttk's fill kernel (dev.zeros)
at::Tensor zeros(const at::Tensor &like, std::vector<int64_t> shape) {
  at::Tensor out = at::empty(shape, like.options());
  if (out.numel()) check(g_fill(g_stream, out.data_ptr<double>(), out.numel(), 0.0), "fill");
  return out;
}

// ttk_env_update's block descriptor (include/ttk.h ttk_env_block, same layout)
struct EnvBlock {
  const double *phi, *x, *A, *y;
  double *out;
  int64_t phi_shape[3], x_shape[3], A_shape[4], y_shape[3];
  int64_t a_strides[4];
};
using env_fn = int (*)(void *, int, int, const EnvBlock *);

// all environment updates of one core step (tt_als.env_update_many): the outputs allocated and the
// descriptors packed here, then ONE ttk_env_update call (fn = its address, ctx = the context)
std::vector<at::Tensor> env_update(int64_t fn, int64_t ctx, bool backward,
                                   const std::vector<std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor>> &items) {
  const size_t n = items.size();
  std::vector<EnvBlock> blocks(n);
  std::vector<at::Tensor> outs;
  outs.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    const at::Tensor &P = std::get<0>(items[i]), &x = std::get<1>(items[i]), &A = std::get<2>(items[i]),
                     &y = std::get<3>(items[i]);
    TORCH_CHECK(P.dim() == 3 && x.dim() == 3 && A.dim() == 4 && y.dim() == 3, "env_update: operand ranks");
    at::Tensor o = backward ? at::empty({x.size(0), A.size(0), y.size(0)}, P.options())
                            : at::empty({x.size(2), A.size(3), y.size(2)}, P.options());
    EnvBlock &e = blocks[i];
    e.phi = P.data_ptr<double>();
    e.x = x.data_ptr<double>();
    e.A = A.data_ptr<double>();
    e.y = y.data_ptr<double>();
    e.out = o.data_ptr<double>();
    for (int k = 0; k < 3; ++k) {
      e.phi_shape[k] = P.size(k);
      e.x_shape[k] = x.size(k);
      e.y_shape[k] = y.size(k);
    }
    for (int k = 0; k < 4; ++k) {
      e.A_shape[k] = A.size(k);
      e.a_strides[k] = A.stride(k);
    }
    outs.push_back(o);
  }
  check(reinterpret_cast<env_fn>(fn)(reinterpret_cast<void *>(ctx), backward ? 1 : 0, (int)n, blocks.data()),
        "env_update");
  return outs;
}

// Tensor metadata helpers that keep the GIL: torch's own Python bindings release it around every
// op (torch.empty, Tensor.view / .t / .permute), which costs ~2 us per call and, with a second
// solve thread in the process, a GIL hand-over each time (2-2.5x per call, tools/gil_bench.py).
at::Tensor empty(const at::Tensor &like, std::vector<int64_t> shape) { return at::empty(shape, like.options()); }

at::Tensor view(const at::Tensor &t, std::vector<int64_t> shape) { return t.view(shape); }

at::Tensor transpose2(const at::Tensor &t) { return t.t(); }

at::Tensor permute(const at::Tensor &t, std::vector<int64_t> dims) { return t.permute(dims); }

#include "ttk_host_eig.inc"

}  // namespace

void set_release_gil(bool on) { g_release_gil = on; }

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("set_release_gil", &set_release_gil);
  m.def("bind", &bind);
  m.def("einsum", &einsum);
  m.def("copy_", &copy_);
  m.def("mul_", &mul_);
  m.def("bind2", &bind2);
  m.def("einsum_cols", &einsum_cols);
  m.def("env_update", &env_update);
  m.def("axpby", &axpby);
  m.def("normalized", &normalized);
  m.def("scale_axis_ss", &scale_axis_ss);
  m.def("dot_into", &dot_into);
  m.def("zeros", &zeros);
  m.def("empty", &empty);
  m.def("view", &view);
  m.def("t", &transpose2);
  m.def("permute", &permute);
  m.def("bind_eig", &eig::bind_eig);
  m.def("eig_als", &eig::eig_als);
  m.def("legacy_randn", &eig::legacy_randn);
  m.def("prune_singular_vals", &eig::prune_singular_vals);
}
