// C-ABI test: one local KKT solve driven through include/ttk.h alone (no Python, no torch), on two
// library contexts with two HIP streams from two host threads at the same time.
//
//   test_abi <fixture>      (tests/golden/abi_lgmres.bin, made by tests/golden/make_abi_fixture.py)
//
// Per thread: create a context, build the Schur-reduced operator on it (ttk_schur_build, the
// `MatVecWrapper` of cy_src/lgmres_cy.pyx:203-331) from the fixture's blocks, solve with the
// whole-solve PETSc LGMRES (ttk_lgmres, src/tt_ipm.py:101-162), copy the solution back.
// Round 1 (default knobs on both contexts): both solutions bit-identical, the iteration count equals
// the oracle's, the solution matches the oracle's PETSc-LGMRES restatement to 1e-8 relative.
// Round 2 (knob isolation): the second context switches its LGMRES steps to the multi-workgroup
// kernels (TTK_KNOB_LGMRES_MW_MIN = 0, another summation order) while the first runs concurrently
// with its defaults: the first context's solution must stay bit-identical to round 1, the second
// must still match the oracle to 1e-8.  Exit 0 = pass.
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/ttk.h"

namespace {

struct Fixture {
  int64_t r, n, R, s, its, m, restart, augment;
  std::vector<double> L[4], A[4], Q[4], invI, b, x;
};

bool load(const char *path, Fixture &f) {
  FILE *fp = std::fopen(path, "rb");
  if (!fp) return false;
  int64_t h[8];
  if (std::fread(h, sizeof(int64_t), 8, fp) != 8) return false;
  f.r = h[0], f.n = h[1], f.R = h[2], f.s = h[3], f.its = h[4], f.m = h[5], f.restart = h[6], f.augment = h[7];
  auto rd = [&](std::vector<double> &v, int64_t cnt) {
    v.resize(cnt);
    return std::fread(v.data(), sizeof(double), cnt, fp) == (size_t)cnt;
  };
  bool ok = true;
  for (int k = 0; k < 4; ++k)
    ok = ok && rd(f.L[k], f.r * f.s * f.r) && rd(f.A[k], f.s * f.n * f.n * f.s) && rd(f.Q[k], f.R * f.s * f.R);
  ok = ok && rd(f.invI, f.m) && rd(f.b, 2 * f.m) && rd(f.x, 2 * f.m);
  std::fclose(fp);
  return ok;
}

double *upload(const std::vector<double> &v, hipStream_t st) {
  double *d = nullptr;
  if (hipMalloc(reinterpret_cast<void **>(&d), v.size() * sizeof(double)) != hipSuccess) return nullptr;
  if (hipMemcpyAsync(d, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess) return nullptr;
  return d;
}

// ttk_einsum descriptor of the local apply 'lsr,smnS,LSR,rnR->lmL' (x patched per application)
void apply_desc(int64_t *d, const double *P, const double *A, const double *Q, const Fixture &f) {
  int64_t k = 0;
  d[k++] = 4 | 256;
  const int64_t r = f.r, n = f.n, R = f.R, s = f.s;
  const int64_t recs[3][9] = {{3, r, s, r, s * r, r, 1, 0, 0},
                              {4, s, n, n, s, n * n * s, n * s, s, 1},
                              {3, R, s, R, s * R, R, 1, 0, 0}};
  const double *ptr[3] = {P, A, Q};
  for (int o = 0; o < 3; ++o) {
    d[k++] = reinterpret_cast<int64_t>(ptr[o]);
    const int nd = (int)recs[o][0];
    d[k++] = nd;
    for (int i = 0; i < 2 * nd; ++i) d[k++] = recs[o][1 + i];
  }
  const int64_t xrec[9] = {0, 3, r, n, R, n * R, R, 1, 0};
  for (int i = 0; i < 9; ++i) d[k++] = xrec[i];
}

struct Result {
  int rc = -1;
  ttk_lgmres_info info{};
  std::vector<double> x;
  char err[256] = "";
};

void solve(const Fixture &f, Result &out, int mw_min) {
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return;
  ttk_ctx ctx = nullptr;
  if ((out.rc = ttk_ctx_create(st, &ctx))) return;
  if (mw_min >= 0 && (out.rc = ttk_ctx_set_knob(ctx, TTK_KNOB_LGMRES_MW_MIN, mw_min, nullptr))) return;
  double *L[4], *A[4], *Q[4];
  for (int k = 0; k < 4; ++k) {
    L[k] = upload(f.L[k], st);
    A[k] = upload(f.A[k], st);
    Q[k] = upload(f.Q[k], st);
  }
  double *invI = upload(f.invI, st), *b = upload(f.b, st), *x = nullptr;
  (void)hipMalloc(reinterpret_cast<void **>(&x), 2 * f.m * sizeof(double));
  const int order[5] = {0, 1, 2, 3, 1};  // B00, B01, B21, B22, B01^T (MatVecWrapper's block order)
  std::vector<int64_t> desc(5 * 36);
  for (int i = 0; i < 5; ++i) apply_desc(desc.data() + 36 * i, L[order[i]], A[order[i]], Q[order[i]], f);
  (void)hipStreamSynchronize(st);
  int64_t h = 0;
  out.rc = ttk_schur_build(ctx, 0, f.m, desc.data(), invI, &h);
  if (!out.rc && h == 0) out.rc = -2;  // operator not representable as a native handle
  if (!out.rc)
    out.rc = ttk_lgmres(ctx, h, b, x, 2 * f.m, (int)f.restart, (int)f.augment, 1e-5, 300, 8, &out.info);
  if (out.rc) std::snprintf(out.err, sizeof(out.err), "%s", ttk_last_error());
  out.x.resize(2 * f.m);
  // the solve's last kernels are still queued on the context's (non-blocking) stream: copy on it
  (void)hipMemcpyAsync(out.x.data(), x, 2 * f.m * sizeof(double), hipMemcpyDeviceToHost, st);
  (void)hipStreamSynchronize(st);
  ttk_schur_free(ctx, h);
  for (int k = 0; k < 4; ++k) {
    (void)hipFree(L[k]);
    (void)hipFree(A[k]);
    (void)hipFree(Q[k]);
  }
  (void)hipFree(invI);
  (void)hipFree(b);
  (void)hipFree(x);
  ttk_ctx_destroy(ctx);
  (void)hipStreamDestroy(st);
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s fixture\n", argv[0]);
    return 2;
  }
  Fixture f;
  if (!load(argv[1], f)) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  auto rel_err = [&](const Result &r) {
    double num = 0.0, den = 0.0;
    for (size_t i = 0; i < f.x.size(); ++i) {
      num = std::fmax(num, std::fabs(r.x[i] - f.x[i]));
      den = std::fmax(den, std::fabs(f.x[i]));
    }
    return num / den;
  };
  auto report = [&](const char *tag, const Result *res) {
    int fail = 0;
    for (int i = 0; i < 2; ++i) {
      std::printf("%s ctx %d: rc %d reason %d its %d res %.6e matvecs %d rel.err %.3e %s\n", tag, i, res[i].rc,
                  res[i].info.reason, res[i].info.its, res[i].info.res, res[i].info.matvecs,
                  res[i].rc ? 0.0 : rel_err(res[i]), res[i].err);
      if (res[i].rc) fail = 1;
    }
    return fail;
  };
  Result res[2];
  {
    std::thread t0(solve, std::cref(f), std::ref(res[0]), -1), t1(solve, std::cref(f), std::ref(res[1]), -1);
    t0.join();
    t1.join();
  }
  if (report("round 1", res)) return 1;
  if (std::memcmp(res[0].x.data(), res[1].x.data(), res[0].x.size() * sizeof(double)) != 0) {
    std::printf("FAIL: the two contexts' solutions differ\n");
    return 1;
  }
  std::printf("its %d (oracle %lld), max |x - x_oracle| / max |x_oracle| = %.3e\n", res[0].info.its,
              (long long)f.its, rel_err(res[0]));
  if (res[0].info.its != f.its || !(rel_err(res[0]) <= 1e-8)) {
    std::printf("FAIL\n");
    return 1;
  }
  Result iso[2];
  {
    std::thread t0(solve, std::cref(f), std::ref(iso[0]), -1), t1(solve, std::cref(f), std::ref(iso[1]), 0);
    t0.join();
    t1.join();
  }
  if (report("round 2", iso)) return 1;
  if (std::memcmp(iso[0].x.data(), res[0].x.data(), res[0].x.size() * sizeof(double)) != 0) {
    std::printf("FAIL: a knob set on another context changed this context's solution\n");
    return 1;
  }
  const bool moved = std::memcmp(iso[1].x.data(), res[0].x.data(), res[0].x.size() * sizeof(double)) != 0;
  std::printf("knob context: summation order %s, its %d\n", moved ? "changed (bits differ)" : "bits unchanged",
              iso[1].info.its);
  if (!(rel_err(iso[1]) <= 1e-8)) {
    std::printf("FAIL: the knob context's solution left the oracle's\n");
    return 1;
  }
  std::printf("PASS\n");
  return 0;
}
