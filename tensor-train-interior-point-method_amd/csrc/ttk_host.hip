// TT-level entry points composed from the library's own kernels: the host-side
// orchestration that the Python layer would otherwise run, behind the C ABI so a reference-side
// caller (Cython / ctypes) reaches the whole operation in one call.  Every step issues the same
// kernel launches with the same shapes, strides and plans as the Python path, so the results are
// bit-identical to it (tests/test_gpu_abi.py).
#include <cmath>
#include <tuple>
#include <cstring>
#include <vector>

#include "ttk_common.h"
#include "ttk_internal.h"

namespace {

// Stream-ordered scratch released when the call returns.  With a capacity (in doubles) it is one
// hipMallocAsync carved into 256-byte slots: an allocation per buffer costs the host several us each,
// which lands on the critical path right after a host read, while the device waits.  A request past
// the capacity gets its own allocation, so the capacity is a hint, never a correctness bound.
struct Scratch {
  hipStream_t st;
  std::vector<void *> ptrs;
  double *base = nullptr;
  int64_t cap = 0, used = 0;
  static int64_t slot(int64_t n) { return ((n > 0 ? n : 1) + 31) & ~(int64_t)31; }
  explicit Scratch(hipStream_t s, int64_t capacity = 0) : st(s) {
    void *p = nullptr;
    if (capacity > 0 && hipMallocAsync(&p, (size_t)capacity * sizeof(double), st) == hipSuccess) {
      ptrs.push_back(p);
      base = static_cast<double *>(p);
      cap = capacity;
    }
  }
  double *get(int64_t n) {
    if (base && used + slot(n) <= cap) {
      double *p = base + used;
      used += slot(n);
      return p;
    }
    void *p = nullptr;
    if (hipMallocAsync(&p, (size_t)(n > 0 ? n : 1) * sizeof(double), st) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return static_cast<double *>(p);
  }
  ~Scratch() {
    for (void *p : ptrs) (void)hipFreeAsync(p, st);
  }
};

struct View {
  const double *p;
  int nd;
  int64_t sh[4], st[4];
};

View mat(const double *p, int64_t rows, int64_t cols) { return View{p, 2, {rows, cols}, {cols, 1}}; }

// ttk_einsum on views, fresh contiguous output (dev.einsum with out=None, fused=False)
int einsum(hipStream_t st, const char *eq, std::initializer_list<View> ops, double *out) {
  int64_t d[1 + 8 * 10 + 1];
  int k = 0;
  d[k++] = (int64_t)ops.size();
  for (const View &o : ops) {
    d[k++] = reinterpret_cast<int64_t>(o.p);
    d[k++] = o.nd;
    for (int i = 0; i < o.nd; ++i) d[k++] = o.sh[i];
    for (int i = 0; i < o.nd; ++i) d[k++] = o.st[i];
  }
  d[k++] = 0;
  return ttk_einsum(st, eq, d, out, 1.0, 0.0);
}

// contiguous copy of a 2-D strided view (dev.clone)
int copy2(hipStream_t st, const double *src, int64_t rows, int64_t cols, int64_t s0, int64_t s1, double *dst) {
  const int64_t shape[2] = {rows, cols}, ss[2] = {s0, s1}, ds[2] = {cols, 1};
  return ttk_copy_nd(st, src, dst, 2, shape, ss, ds, 1.0, 0.0);
}

// `prune_singular_vals` (cy_src/tt_ops_cy.pyx:161-177) / the tracked variant of the PSD and mask
// roundings (:261-388): sc[i] = sum_{j>=i} s_j^2 accumulated from the end as np.cumsum does.
int truncation_rank(const std::vector<double> &s, double eps, bool track, double *tail) {
  const int k = (int)s.size();
  *tail = 0.0;
  if (!track) {
    bool zero = true;
    for (double v : s) zero = zero && v == 0.0;
    if (zero) return 1;
  }
  std::vector<double> sc(k);
  double acc = 0.0;
  for (int i = k - 1; i >= 0; --i) {
    acc += std::fabs(s[i]) * std::fabs(s[i]);
    sc[i] = acc;
  }
  const double e2 = eps * eps;
  int r = 0;
  for (int i = 0; i < k; ++i)
    if (sc[i] < e2) {
      r = i;
      break;
    }
  r = r < 1 ? 1 : r;
  if (sc[k - 1] > e2) r = k;
  if (track && r < k) *tail = sc[r];
  return r;
}

View v3(const double *p, int64_t a, int64_t b, int64_t c) { return View{p, 3, {a, b, c}, {b * c, c, 1}}; }

// einsum with an explicit (strided) output view and alpha / beta (dev.einsum(..., out=view))
int einsum_out(hipStream_t st, const char *eq, std::initializer_list<View> ops, double *out, int ond,
               const int64_t *ost, double alpha, double beta) {
  int64_t d[1 + 8 * 10 + 2 + 8];
  int k = 0;
  d[k++] = (int64_t)ops.size();
  for (const View &o : ops) {
    d[k++] = reinterpret_cast<int64_t>(o.p);
    d[k++] = o.nd;
    for (int i = 0; i < o.nd; ++i) d[k++] = o.sh[i];
    for (int i = 0; i < o.nd; ++i) d[k++] = o.st[i];
  }
  d[k++] = 1;
  d[k++] = ond;
  for (int i = 0; i < ond; ++i) d[k++] = ost[i];
  return ttk_einsum(st, eq, d, out, alpha, beta);
}

}  // namespace

extern "C" {

int ttk_dense_schur_solve(ttk_ctx ctx, int64_t r, int64_t n, int64_t R, const ttk_local_block *blk,
                          const double *rhs, const double *inv_I, double *sol, double *rcond_out) {
  ttk::CtxScope scope(ctx);
  hipStream_t st = ttk::ctx().stream;
  if (rcond_out) *rcond_out = NAN;
  const int64_t m = r * n * R;
  if (r < 1 || n < 1 || R < 1 || !blk || !rhs || !inv_I || !sol || m > (1 << 20)) {
    ttk::set_error("ttk_dense_schur_solve: bad arguments");
    return TTK_ERR_ARG;
  }
  static const char *ASSEMBLE = "lsr,smnS,LSR->lmLrnR", *APPLY = "lsr,smnS,LSR,rnR->lmL",
                    *APPLY_T = "lsr,smnS,LSR,lmL->rnR", *MATMUL = "ik,kj->ij";
  enum { B00, B01, B21, B22 };
  auto ops3 = [&](int b) {
    const ttk_local_block &q = blk[b];
    return std::make_tuple(v3(q.L, r, q.s, r),
                           View{q.A, 4, {q.s, n, n, q.S}, {q.a_strides[0], q.a_strides[1], q.a_strides[2], q.a_strides[3]}},
                           v3(q.R, R, q.S, R));
  };
  Scratch sc(st, 7 * Scratch::slot(m) + 5 * Scratch::slot(m * m) + Scratch::slot(2 * m + 16) + Scratch::slot(m / 2 + 1));
  double *rd = sc.get(m), *rc = sc.get(m), *rp = sc.get(m), *LXI = sc.get(m * m), *Leq = sc.get(m * m),
         *LZ = sc.get(m * m), *t = sc.get(m), *bvec = sc.get(m), *T1 = sc.get(m * m), *Am = sc.get(m * m),
         *t2 = sc.get(m), *t3 = sc.get(m), *work = sc.get(2 * m + 16);
  int *piv = reinterpret_cast<int *>(sc.get(m / 2 + 1));
  if (!rd || !rc || !rp || !LXI || !Leq || !LZ || !t || !bvec || !T1 || !Am || !t2 || !t3 || !work || !piv) {
    ttk::set_error("ttk_dense_schur_solve: scratch allocation failed");
    return TTK_ERR_HIP;
  }
  const int64_t sh3[3] = {r, n, R}, st_blk[3] = {3 * n * R, R, 1}, st_c[3] = {n * R, R, 1};
  const int64_t out6[6] = {n * R * m, R * m, m, n * R, R, 1};
  const int64_t mm[2] = {m, m}, s_mat[2] = {m, 1}, s_row[2] = {0, 1}, out2[2] = {1, 1};
  auto col = [&](int j) { return rhs + j * n * R; };  // rhs[:, j] as (r, n, R) view, strides st_blk
  int rc_ = TTK_OK;
#define STEP(x)              \
  do {                       \
    if (rc_ == TTK_OK) rc_ = (x); \
  } while (0)
  STEP(ttk_copy_nd(st, col(1), rd, 3, sh3, st_blk, st_c, 1.0, 0.0));
  STEP(ttk_copy_nd(st, col(2), rc, 3, sh3, st_blk, st_c, 1.0, 0.0));
  STEP(ttk_copy_nd(st, col(0), rp, 3, sh3, st_blk, st_c, 1.0, 0.0));
  {
    auto [a, b, c] = ops3(B22);
    STEP(einsum(st, ASSEMBLE, {a, b, c}, LXI));
  }
  STEP(ttk_mul_nd(st, LXI, inv_I, LXI, 2, mm, s_mat, s_row, s_mat, 1.0, 0.0));  // LXI * inv_I[col]
  {
    auto [a, b, c] = ops3(B01);
    STEP(einsum(st, ASSEMBLE, {a, b, c}, Leq));
  }
  {
    auto [a, b, c] = ops3(B21);
    STEP(einsum(st, ASSEMBLE, {a, b, c}, LZ));
  }
  if (rc_) return rc_;
  rc_ = ttk_cholesky_sync(st, LZ, (int)m);
  if (rc_) return rc_;  // TTK_ERR_NOT_PD: scipy's LinAlgError -> the caller's iterative fallback
  STEP(hipMemcpyAsync(t, rc, m * sizeof(double), hipMemcpyDeviceToDevice, st) ? TTK_ERR_HIP : 0);
  STEP(einsum_out(st, MATMUL, {mat(LXI, m, m), mat(rd, m, 1)}, t, 2, out2, -1.0, 1.0));
  STEP(ttk_trsm_lower(st, LZ, (int)m, t, 1, 1, 0));
  STEP(ttk_trsm_lower(st, LZ, (int)m, t, 1, 1, 1));
  STEP(hipMemcpyAsync(bvec, rp, m * sizeof(double), hipMemcpyDeviceToDevice, st) ? TTK_ERR_HIP : 0);
  STEP(einsum_out(st, MATMUL, {mat(Leq, m, m), mat(t, m, 1)}, bvec, 2, out2, -1.0, 1.0));
  STEP(ttk_trsm_lower(st, LZ, (int)m, LXI, (int)m, (int)m, 0));
  STEP(ttk_trsm_lower(st, LZ, (int)m, LXI, (int)m, (int)m, 1));
  STEP(einsum(st, MATMUL, {mat(LXI, m, m), View{Leq, 2, {m, m}, {1, m}}}, T1));
  STEP(einsum(st, MATMUL, {mat(Leq, m, m), mat(T1, m, m)}, Am));
  {
    auto [a, b, c] = ops3(B00);
    STEP(einsum_out(st, ASSEMBLE, {a, b, c}, Am, 6, out6, 1.0, 1.0));
  }
  STEP(ttk_add_diag(st, Am, (int)m, (int)m, 1e-11));
  if (rc_) return rc_;
  // getrf here; its dgecon estimate runs on the context's side stream while the back-substitutions
  // below proceed speculatively (their result is discarded when the status or rcond rejects the
  // factors, as the early returns of the step-by-step path would have) -- one host read at the end
  int forked = 0;
  rc_ = ttk::lu_factor_fork_rcond(st, Am, (int)m, piv, work, &forked);
  if (rc_) return rc_;
  STEP(ttk_lu_solve(st, Am, (int)m, piv, bvec, 1, 1));
  double *s0 = sol, *s1 = sol + n * R, *s2 = sol + 2 * n * R;  // sol[:, j] views, strides st_blk
  STEP(ttk_copy_nd(st, bvec, s0, 3, sh3, st_c, st_blk, 1.0, 0.0));
  STEP(hipMemcpyAsync(t2, rd, m * sizeof(double), hipMemcpyDeviceToDevice, st) ? TTK_ERR_HIP : 0);
  {
    auto [a, b, c] = ops3(B01);
    const View x{s0, 3, {r, n, R}, {st_blk[0], st_blk[1], st_blk[2]}};
    STEP(einsum_out(st, APPLY_T, {a, b, c, x}, t2, 3, st_c, -1.0, 1.0));
  }
  STEP(ttk_mul_nd(st, t2, inv_I, s2, 3, sh3, st_c, st_c, st_blk, 1.0, 0.0));
  STEP(hipMemcpyAsync(t3, rc, m * sizeof(double), hipMemcpyDeviceToDevice, st) ? TTK_ERR_HIP : 0);
  {
    auto [a, b, c] = ops3(B22);
    const View x{s2, 3, {r, n, R}, {st_blk[0], st_blk[1], st_blk[2]}};
    STEP(einsum_out(st, APPLY, {a, b, c, x}, t3, 3, st_c, -1.0, 1.0));
  }
  STEP(ttk_trsm_lower(st, LZ, (int)m, t3, 1, 1, 0));
  STEP(ttk_trsm_lower(st, LZ, (int)m, t3, 1, 1, 1));
  STEP(ttk_copy_nd(st, t3, s1, 3, sh3, st_c, st_blk, 1.0, 0.0));
#undef STEP
  if (forked && ttk::lu_rcond_join(st)) return TTK_ERR_HIP;
  int lu_info = 0;
  double rcond = 0.0;
  if (hipMemcpyAsync(&lu_info, ttk::ctx().status, sizeof(int), hipMemcpyDeviceToHost, st) ||
      hipMemcpyAsync(&rcond, ttk::ctx().rcond, sizeof(double), hipMemcpyDeviceToHost, st))
    return TTK_ERR_HIP;
  ttk::note_sync();
  if (hipStreamSynchronize(st)) return TTK_ERR_HIP;
  if (rcond_out) *rcond_out = rcond;
  if (lu_info) {
    ttk::set_error("Matrix is singular (zero pivot at %d).", lu_info);
    return TTK_ERR_SINGULAR;
  }
  if (rcond < 0.5 * 2.220446049250313e-16) return TTK_ILL_CONDITIONED;  // LinAlgWarning as an error
  return rc_;
}

int ttk_dense_schur_solve_ineq(ttk_ctx ctx, int64_t r, int64_t n, int64_t R, const ttk_local_block *blk,
                               const double *rhs, const double *inv_I, double *sol) {
  ttk::CtxScope scope(ctx);
  hipStream_t st = ttk::ctx().stream;
  const int64_t m = r * n * R;
  if (r < 1 || n < 1 || R < 1 || !blk || !rhs || !inv_I || !sol || m > (1 << 20)) {
    ttk::set_error("ttk_dense_schur_solve_ineq: bad arguments");
    return TTK_ERR_ARG;
  }
  static const char *ASSEMBLE = "lsr,smnS,LSR->lmLrnR", *APPLY = "lsr,smnS,LSR,rnR->lmL",
                    *APPLY_T = "lsr,smnS,LSR,lmL->rnR", *MATMUL = "ik,kj->ij";
  enum { B00, B01, B21, B22, B31, B33 };
  auto ops3 = [&](int b) {
    const ttk_local_block &q = blk[b];
    return std::make_tuple(v3(q.L, r, q.s, r),
                           View{q.A, 4, {q.s, n, n, q.S}, {q.a_strides[0], q.a_strides[1], q.a_strides[2], q.a_strides[3]}},
                           v3(q.R, R, q.S, R));
  };
  Scratch sc(st, 12 * Scratch::slot(m) + 12 * Scratch::slot(m * m) + Scratch::slot(2 * m + 16) +
                     2 * Scratch::slot(m / 2 + 1));
  double *rp = sc.get(m), *rd = sc.get(m), *rc = sc.get(m), *rt = sc.get(m), *LZ = sc.get(m * m),
         *LZ_rc = sc.get(m), *LZ_LX = sc.get(m * m), *Leq = sc.get(m * m), *Top = sc.get(m * m),
         *LZ_LXI = sc.get(m * m), *w = sc.get(m), *u = sc.get(m), *v = sc.get(m), *Am = sc.get(m * m),
         *T = sc.get(m * m), *Dm = sc.get(m * m), *TL = sc.get(m * m), *Top2 = sc.get(m * m), *Leq2 = sc.get(m * m),
         *Dv = sc.get(m), *DT = sc.get(m * m), *y = sc.get(m), *t2 = sc.get(m), *t3 = sc.get(m),
         *work = sc.get(2 * m + 16);
  int *dpiv = reinterpret_cast<int *>(sc.get(m / 2 + 1)), *piv = reinterpret_cast<int *>(sc.get(m / 2 + 1));
  for (double *p : {rp, rd, rc, rt, LZ, LZ_rc, LZ_LX, Leq, Top, LZ_LXI, w, u, v, Am, T, Dm, TL, Top2, Leq2, Dv, DT, y,
                    t2, t3, work})
    if (!p || !dpiv || !piv) {
      ttk::set_error("ttk_dense_schur_solve_ineq: scratch allocation failed");
      return TTK_ERR_HIP;
    }
  const int64_t sh3[3] = {r, n, R}, st_blk[3] = {4 * n * R, R, 1}, st_c[3] = {n * R, R, 1};
  const int64_t mm[2] = {m, m}, s_mat[2] = {m, 1}, s_row[2] = {0, 1}, out1[2] = {1, 1}, outm[2] = {m, 1};
  const View LeqT{Leq, 2, {m, m}, {1, m}};
  auto col = [&](int j) { return rhs + j * n * R; };  // rhs[:, j] as (r, n, R) view, strides st_blk
  auto dcopy = [&](double *dst, const double *src, int64_t len) {
    return hipMemcpyAsync(dst, src, len * sizeof(double), hipMemcpyDeviceToDevice, st) ? TTK_ERR_HIP : TTK_OK;
  };
  auto assemble = [&](int b, double *out) {
    auto [a, bb, c] = ops3(b);
    return einsum(st, ASSEMBLE, {a, bb, c}, out);
  };
  auto fbsub = [&](double *B, int nrhs) {  // forward_backward_sub, src/tt_ipm.py:178-181
    int e = ttk_trsm_lower(st, LZ, (int)m, B, nrhs, nrhs, 0);
    return e ? e : ttk_trsm_lower(st, LZ, (int)m, B, nrhs, nrhs, 1);
  };
  int rc_ = TTK_OK;
#define STEP(x)                   \
  do {                            \
    if (rc_ == TTK_OK) rc_ = (x); \
  } while (0)
  // the statement order of _ipm_local_solver_ineq's dense branch (src/tt_ipm.py:303-352)
  STEP(assemble(B21, LZ));
  if (rc_) return rc_;
  rc_ = ttk_cholesky_sync(st, LZ, (int)m);
  if (rc_) return rc_;  // TTK_ERR_NOT_PD: LinAlgError -> the caller's iterative fallback
  STEP(ttk_copy_nd(st, col(0), rp, 3, sh3, st_blk, st_c, 1.0, 0.0));
  STEP(ttk_copy_nd(st, col(1), rd, 3, sh3, st_blk, st_c, 1.0, 0.0));
  STEP(ttk_copy_nd(st, col(2), rc, 3, sh3, st_blk, st_c, 1.0, 0.0));
  STEP(ttk_copy_nd(st, col(3), rt, 3, sh3, st_blk, st_c, 1.0, 0.0));
  STEP(dcopy(LZ_rc, rc, m));
  STEP(fbsub(LZ_rc, 1));
  STEP(assemble(B22, LZ_LX));
  STEP(fbsub(LZ_LX, (int)m));
  STEP(assemble(B01, Leq));
  STEP(assemble(B31, Top));
  STEP(ttk_mul_nd(st, LZ_LX, inv_I, LZ_LXI, 2, mm, s_mat, s_row, s_mat, 1.0, 0.0));  // LZ_LX * inv_I[col]
  STEP(dcopy(w, LZ_rc, m));
  STEP(einsum_out(st, MATMUL, {mat(LZ_LXI, m, m), mat(rd, m, 1)}, w, 2, out1, -1.0, 1.0));
  STEP(dcopy(u, rp, m));
  STEP(einsum_out(st, MATMUL, {mat(Leq, m, m), mat(w, m, 1)}, u, 2, out1, -1.0, 1.0));
  STEP(dcopy(v, rt, m));
  STEP(einsum_out(st, MATMUL, {mat(Top, m, m), mat(w, m, 1)}, v, 2, out1, -1.0, 1.0));
  STEP(assemble(B00, Am));
  STEP(einsum(st, MATMUL, {mat(LZ_LXI, m, m), LeqT}, T));
  STEP(einsum_out(st, MATMUL, {mat(Leq, m, m), mat(T, m, m)}, Am, 2, outm, 1.0, 1.0));
  STEP(assemble(B33, Dm));
  STEP(einsum_out(st, MATMUL, {mat(Top, m, m), mat(LZ_LX, m, m)}, Dm, 2, outm, 1.0, 1.0));
  STEP(ttk_add_diag(st, Dm, (int)m, (int)m, 1e-11));
  STEP(einsum(st, MATMUL, {mat(Top, m, m), mat(LZ_LXI, m, m)}, TL));
  STEP(einsum(st, MATMUL, {mat(TL, m, m), LeqT}, Top2));
  STEP(einsum(st, MATMUL, {mat(Leq, m, m), mat(LZ_LX, m, m)}, Leq2));
  if (rc_) return rc_;
  double rcond = 0.0;  // scipy.linalg.lu_factor: no condition check (src/tt_ipm.py:330)
  rc_ = ttk_lu_sync(st, Dm, (int)m, dpiv, work, &rcond);
  if (rc_) return rc_;  // TTK_ERR_SINGULAR
  STEP(dcopy(Dv, v, m));
  STEP(ttk_lu_solve(st, Dm, (int)m, dpiv, Dv, 1, 1));
  STEP(einsum_out(st, MATMUL, {mat(Leq2, m, m), mat(Dv, m, 1)}, u, 2, out1, -1.0, 1.0));
  STEP(dcopy(DT, Top2, m * m));
  STEP(ttk_lu_solve(st, Dm, (int)m, dpiv, DT, (int)m, (int)m));
  STEP(einsum_out(st, MATMUL, {mat(Leq2, m, m), mat(DT, m, m)}, Am, 2, outm, -1.0, 1.0));
  if (rc_) return rc_;
  rc_ = ttk_lu_sync(st, Am, (int)m, piv, work, &rcond);
  if (rc_) return rc_;
  STEP(dcopy(y, u, m));
  STEP(ttk_lu_solve(st, Am, (int)m, piv, y, 1, 1));
  double *s0 = sol, *s1 = sol + n * R, *s2 = sol + 2 * n * R, *s3 = sol + 3 * n * R;  // sol[:, j], strides st_blk
  STEP(ttk_copy_nd(st, y, s0, 3, sh3, st_c, st_blk, 1.0, 0.0));
  STEP(einsum_out(st, MATMUL, {mat(Top2, m, m), mat(y, m, 1)}, v, 2, out1, -1.0, 1.0));
  STEP(ttk_lu_solve(st, Dm, (int)m, dpiv, v, 1, 1));
  STEP(ttk_copy_nd(st, v, s3, 3, sh3, st_c, st_blk, 1.0, 0.0));
  STEP(dcopy(t2, rd, m));
  {
    auto [a, b, c] = ops3(B01);
    const View x{s0, 3, {r, n, R}, {st_blk[0], st_blk[1], st_blk[2]}};
    STEP(einsum_out(st, APPLY_T, {a, b, c, x}, t2, 3, st_c, -1.0, 1.0));
  }
  STEP(ttk_mul_nd(st, t2, inv_I, s2, 3, sh3, st_c, st_c, st_blk, 1.0, 0.0));
  STEP(ttk_copy_nd(st, s3, s2, 3, sh3, st_blk, st_blk, -1.0, 1.0));
  STEP(dcopy(t3, rc, m));
  {
    auto [a, b, c] = ops3(B22);
    const View x{s2, 3, {r, n, R}, {st_blk[0], st_blk[1], st_blk[2]}};
    STEP(einsum_out(st, APPLY, {a, b, c, x}, t3, 3, st_c, -1.0, 1.0));
  }
  STEP(fbsub(t3, 1));
  STEP(ttk_copy_nd(st, t3, s1, 3, sh3, st_c, st_blk, 1.0, 0.0));
#undef STEP
  return rc_;
}

int ttk_round(ttk_ctx ctx, int d, double *const *cores, const int64_t *inner, int64_t *ranks, double eps, int mode,
              double *tail_out) {
  ttk::CtxScope scope(ctx);
  hipStream_t st = ttk::ctx().stream;
  if (tail_out) *tail_out = NAN;
  if (d < 1 || !cores || !inner || !ranks || (mode != 0 && mode != 1) || ranks[0] != 1 || ranks[d] != 1) {
    ttk::set_error("ttk_round: bad arguments");
    return TTK_ERR_ARG;
  }
  bool all1 = true;
  for (int k = 0; k <= d; ++k) all1 = all1 && ranks[k] == 1;
  if (d == 1 || all1) return TTK_OK;  // tt_rank_reduce returns the train unchanged
  const bool track = mode == 1;
  if (track) eps = eps / 2.0;
  eps = eps / std::sqrt((double)(d - 1));
  std::vector<int64_t> r(ranks, ranks + d + 1);
  // Scratch for the whole call in one allocation (Scratch above), sized up front: the QR sweep's
  // shapes follow from the ranks alone, the SVD sweep's are bounded by them (rank <= r[idx] after
  // the QR sweep).
  int64_t total = 0;
  {
    const auto words = Scratch::slot;
    std::vector<int64_t> q(r);
    for (int i = d - 1; i >= 1; --i) {
      const int64_t m = inner[i] * q[i + 1], n = q[i], k = m < n ? m : n;
      total += words(m * n) + words(m * k) + words(k * n) + words(ttk_qr_work((int)m, (int)n)) +
               words(q[i - 1] * inner[i - 1] * k);
      q[i] = k;
    }
    int64_t rank = 1;
    for (int idx = 0; idx + 1 < d; ++idx) {
      const int64_t n = q[idx + 1], mb = rank * inner[idx], kb = mb < n ? mb : n;
      int64_t wb = 0;
      for (int64_t rr = 1; rr <= rank; ++rr) {
        const int64_t w = ttk_svd_work((int)(rr * inner[idx]), (int)n);
        wb = w > wb ? w : wb;
      }
      total += words(mb * kb) + words(kb) + words(kb * n) + words(wb) + words(kb * inner[idx + 1] * q[idx + 2]);
      rank = kb;
    }
  }
  Scratch sc(st, total);
  bool oom = false;
  auto get = [&](int64_t n) {
    double *p = sc.get(n);
    oom = oom || !p;
    return p;
  };
  int rc = TTK_OK;
  // ---- right-to-left QR sweep (tt_rl_orthogonalise, cy_src/tt_ops_cy.pyx:132-159).  Core i-1's
  // update (cores[i-1] R^T) stays in scratch: the next step and the SVD sweep read it from there
  // and only ever write the core's final value, so no copy back is needed.
  const double *cur = cores[d - 1];
  for (int i = d - 1; i >= 1 && rc == TTK_OK; --i) {
    const int64_t m = inner[i] * r[i + 1], n = r[i], k = m < n ? m : n;
    double *At = get(m * n), *Q = get(m * k), *R = get(k * n), *w = get(ttk_qr_work((int)m, (int)n));
    const int64_t lead = r[i - 1] * inner[i - 1];
    double *prev = get(lead * k);
    if (oom) {
      ttk::set_error("ttk_round: scratch allocation failed");
      return TTK_ERR_HIP;
    }
    // core i as (r_i, n_i R_i) row-major is the unfolding's transpose: the QR kernel takes it, and
    // leaves Q^T (core i's new (k, n_i, R_i)), in that layout; into scratch when it would overwrite
    // its own input.  Shapes the blocked QR takes go through the transposing copies and ttk_qr.
    double *qt = cur == cores[i] ? Q : cores[i];
    rc = ttk::qr_colmajor(st, cur, (int)m, (int)n, qt, R, w);
    if (rc == TTK_OK && qt != cores[i])
      rc = hipMemcpyAsync(cores[i], qt, k * m * sizeof(double), hipMemcpyDeviceToDevice, st) ? TTK_ERR_HIP : 0;
    if (rc == TTK_ERR_ARG) {
      rc = copy2(st, cur, m, n, 1, m, At);  // unfolding (r_i, n_i R_i) transposed
      if (!rc) rc = ttk_qr(st, At, (int)m, (int)n, Q, R, w);
      if (!rc) rc = copy2(st, Q, k, m, 1, k, cores[i]);  // Q^T -> core i (k, n_i, R_i)
    }
    if (!rc) rc = einsum(st, "ij,kj->ik", {mat(cores[i - 1], lead, n), mat(R, k, n)}, prev);
    cur = prev;
    r[i] = k;
  }
  // ---- left-to-right truncated-SVD sweep (cy_src/tt_ops_cy.pyx:200-222); `cur` holds core idx
  double tail = 0.0;
  int64_t rank = 1;
  std::vector<double> s;
  for (int idx = 0; idx + 1 < d && rc == TTK_OK; ++idx) {
    const int64_t m = rank * inner[idx], n = r[idx + 1], k = m < n ? m : n;
    double *U = get(m * k), *S = get(k), *Vt = get(k * n), *w = get(ttk_svd_work((int)m, (int)n));
    const int64_t rest = inner[idx + 1] * r[idx + 2];
    double *nxt = get(k * rest);
    if (oom) {
      ttk::set_error("ttk_round: scratch allocation failed");
      return TTK_ERR_HIP;
    }
    // the singular values reach the host from the SVD kernel's own stores (ttk_svd_tol_read)
    s.assign(k, 0.0);
    rc = ttk_svd_tol_read(st, cur, (int)m, (int)n, U, S, Vt, w, track ? 0.0 : 1e-3 * eps, s.data());
    if (rc) break;
    double t = 0.0;
    const int64_t nr = truncation_rank(s, eps, track, &t);
    tail += t;
    rc = copy2(st, U, m, nr, k, 1, cores[idx]);  // U[:, :nr] -> core idx (rank, n_idx, nr)
    const View sv{S, 1, {nr}, {1}}, vv{Vt, 2, {nr, n}, {n, 1}};
    if (!rc) rc = einsum(st, "r,rj,jk->rk", {sv, vv, mat(cores[idx + 1], n, rest)}, nxt);
    if (!rc && idx + 2 == d)
      rc = hipMemcpyAsync(cores[idx + 1], nxt, nr * rest * sizeof(double), hipMemcpyDeviceToDevice, st) ? TTK_ERR_HIP : 0;
    cur = nxt;
    r[idx + 1] = nr;
    rank = nr;
  }
  if (rc) return rc;
  for (int k = 0; k <= d; ++k) ranks[k] = r[k];
  if (track && tail_out) *tail_out = std::pow(tail, 1.0 / (2 * d));
  return TTK_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- zip-up products (one call)
// `tt_fast_matrix_vec_mul` / `tt_fast_mat_mat_mul` / `tt_fast_hadamard` (cy_src/tt_ops_cy.pyx:
// 391-502) as the device path computes them: the exact core-wise product with
// Kronecker bonds, one einsum per core into the caller's buffer, then ONE rounding at eps
// (ttk_round mode 0, in place).  Same einsum plans and the same rounding launches as
// tt_ops.tt_fast_* in Python, so bit-identical to it.
extern "C" int ttk_zipup(ttk_ctx ctx, int kind, int d, const double *const *a, const int64_t *a_ranks,
                         const double *const *b, const int64_t *b_ranks, const int64_t *modes, double eps,
                         double *const *out, int64_t *out_ranks) {
  ttk::CtxScope scope(ctx);
  hipStream_t st = ttk::ctx().stream;
  if (d < 1 || kind < 0 || kind > 3 || !a || !b || !a_ranks || !b_ranks || !modes || !out || !out_ranks) {
    ttk::set_error("ttk_zipup: bad arguments");
    return TTK_ERR_ARG;
  }
  std::vector<int64_t> inner(d);
  int rc = TTK_OK;
  for (int k = 0; k < d && rc == TTK_OK; ++k) {
    const int64_t ra = a_ranks[k], Ra = a_ranks[k + 1], rb = b_ranks[k], Rb = b_ranks[k + 1];
    const int64_t m0 = modes[3 * k], m1 = modes[3 * k + 1], m2 = modes[3 * k + 2];
    const View A4{a[k], 4, {ra, m0, m1, Ra}, {m0 * m1 * Ra, m1 * Ra, Ra, 1}};
    if (kind == 0) {  // mat (ra, m, n, Ra) x vec (rb, n, Rb) -> (ra rb, m, Ra Rb)
      rc = einsum(st, "amnA,rnR->armAR", {A4, v3(b[k], rb, m1, Rb)}, out[k]);
      inner[k] = m0;
    } else if (kind == 1) {  // (ra, m, k, Ra) x (rb, k, n, Rb) -> (ra rb, m, n, Ra Rb)
      const View B4{b[k], 4, {rb, m1, m2, Rb}, {m1 * m2 * Rb, m2 * Rb, Rb, 1}};
      rc = einsum(st, "amkA,bknB->abmnAB", {A4, B4}, out[k]);
      inner[k] = m0 * m2;
    } else if (kind == 2) {  // vectors (ra, i, Ra) o (rb, i, Rb)
      rc = einsum(st, "aiA,biB->abiAB", {v3(a[k], ra, m0, Ra), v3(b[k], rb, m0, Rb)}, out[k]);
      inner[k] = m0;
    } else {  // matrices (ra, i, j, Ra) o (rb, i, j, Rb)
      const View B4{b[k], 4, {rb, m0, m1, Rb}, {m0 * m1 * Rb, m1 * Rb, Rb, 1}};
      rc = einsum(st, "aijA,bijB->abijAB", {A4, B4}, out[k]);
      inner[k] = m0 * m1;
    }
  }
  for (int k = 0; k <= d; ++k) out_ranks[k] = a_ranks[k] * b_ranks[k];
  if (rc != TTK_OK || d == 1 || !(eps > 0.0)) return rc;  // _kron_round: no rounding
  return ttk_round(ctx, d, out, inner.data(), out_ranks, eps, 0, nullptr);
}
