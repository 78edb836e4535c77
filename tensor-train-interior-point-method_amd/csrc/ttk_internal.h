// Internal (non-ABI) entry points shared between libttk translation units.
#ifndef TTK_INTERNAL_H
#define TTK_INTERNAL_H

#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/ttk.h"

namespace ttk {
inline int env_int(const char *name, int dflt) {
  const char *v = std::getenv(name);
  return v ? std::atoi(v) : dflt;
}
// Per-context state (`ttk_ctx`): every scratch buffer, staging ring and handle table the library
// keeps between calls lives in a context, so two contexts (each with its own stream, driven by its
// own host thread) never share mutable state.  The plan cache (immutable plans + their offset
// tables) is shared and lock-protected.  ctx() is the calling thread's bound context, or the
// process default context when none is bound (the Python host layer's single-stream model).
struct UpSlot {
  double *p = nullptr;
  size_t n = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;
};
constexpr int UP_SLOTS = 64;

struct Ctx {
  hipStream_t stream = nullptr;
  double *scratch = nullptr;  // einsum intermediates (unbatched calls)
  int64_t scratch_n = 0;
  void *batch = nullptr;      // einsum batch recorder (ttk_einsum.hip)
  double *splitk = nullptr;   // split-K partial slabs
  int64_t splitk_n = 0;
  double *dev_scalar = nullptr;
  void *schur = nullptr;      // Schur operator handle table (ttk_einsum.hip)
  double *schur_w = nullptr;
  int64_t schur_wcap = 0;
  unsigned *dep = nullptr;    // in-launch hand-off arrival counter (monotonic; ttk_einsum.hip)
  unsigned dep_total = 0;     // arrivals of every hand-off launch issued on this context so far
  unsigned tick_total = 0;    // workgroup tickets (dep[2]) of every hand-off launch issued so far
  unsigned *splitk_cnt = nullptr;  // per-tile arrival counters of the one-launch split-K GEMM (reset by it)
  unsigned *colr = nullptr;   // per-column round counters of the one-launch Jacobi sweep (ttk_linalg.hip)
  int64_t colr_n = 0;
  double *lgmres = nullptr;   // LGMRES partial sums
  int64_t lgmres_n = 0;
  int *status = nullptr;      // dense factorisation status words
  double *rcond = nullptr;
  double *mapped_h = nullptr, *mapped_d = nullptr;  // host-coherent read buffer
  size_t mapped_n = 0;
  UpSlot up[UP_SLOTS];        // pinned upload ring
  int up_next = 0;
  hipStream_t side = nullptr;  // second stream (dgecon overlapped with the rest of a dense solve)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // numerics knobs (ttk_ctx_set_knob; several change summation order, so they are per context:
  // flipping one on a context never changes another context's results).  Defaults from the
  // environment at context creation.
  int knob[TTK_KNOB_COUNT] = {env_int("TTK_FUSED_APPLY", 1) != 0 ? 1 : 0, env_int("TTK_FUSED_MFMA", 1) != 0 ? 1 : 0,
                              env_int("TTK_SPLITK", 1) != 0 ? 1 : 0,
                              env_int("TTK_SPLITK_MINK", 128) > 0 ? env_int("TTK_SPLITK_MINK", 128) : 128,
                              env_int("TTK_LGMRES_MW_MIN", 16384), env_int("TTK_MFMA_CSPLIT", 1) != 0 ? 1 : 0,
                              env_int("TTK_APPLY_DUAL", 1) != 0 ? 1 : 0, env_int("TTK_RCOND_EXACT", 0) != 0 ? 1 : 0,
                              env_int("TTK_SCHUR_ONE", 1) != 0 ? 1 : 0, env_int("TTK_ARNOLDI_ONE", 0) != 0 ? 1 : 0,
                              env_int("TTK_SCHUR_PREP", 1) != 0 ? 1 : 0, env_int("TTK_SPLITK_FUSED", 1) != 0 ? 1 : 0,
                              env_int("TTK_TRI_HOIST", 1) != 0 ? 1 : 0, env_int("TTK_TRI_ONE", 0),
                              env_int("TTK_SVD_SWEEP_ONE", 0) != 0 ? 1 : 0, env_int("TTK_TRI_PERSIST", 0) != 0 ? 1 : 0,
                              env_int("TTK_SYEV_WAVES8", 1) != 0 ? 1 : 0, env_int("TTK_BT_STAGE", 1) != 0 ? 1 : 0};
};
Ctx &ctx();
Ctx *ctx_swap(Ctx *c);       // bind c to the calling thread, return the previous binding
void schur_release(Ctx &c);  // ttk_einsum.hip: Schur handle table + operand images of a context
// scratch of the bound context at its initial sizes (ttk_ctx_create): split-K slabs, LGMRES partials,
// the Schur operator's w buffer
int presize_splitk();
int presize_lgmres();
int presize_schur();
}  // namespace ttk

struct ttk_ctx_s {
  ttk::Ctx c;
};

namespace ttk {
// binds an ABI context for the duration of a call (NULL: keep the thread's current context)
struct CtxScope {
  Ctx *prev;
  bool on;
  explicit CtxScope(ttk_ctx_s *h) : prev(nullptr), on(h != nullptr) {
    if (on) prev = ctx_swap(&h->c);
  }
  ~CtxScope() {
    if (on) ctx_swap(prev);
  }
};
void ctx_free_einsum(Ctx &c);  // ttk_einsum.hip: batch + Schur tables of a context being destroyed

// ttk_dense.hip: blocked multi-workgroup Cholesky (status = LAPACK info, device int) and
// triangular solve op(L) X = B; both enqueue on `st` without synchronising.
int cholesky_blocked(hipStream_t st, double *A, int n, int *status);
int trsm_blocked(hipStream_t st, const double *L, int n, double *B, int nrhs, int ldb, int trans);
// blocked getrf (device pivots and LAPACK info in `status`) and, if want_rcond, the dgecon
// 1-norm estimate into device `rcond`; work >= n doubles.  Enqueued without synchronising.
int lu_blocked(hipStream_t st, double *A, int n, int *piv, double *work, int *status, double *rcond, int want_rcond);
// want_rcond = 2: the column sums only; the dgecon kernel is then launched by lu_rcond_launch
int lu_rcond_launch(hipStream_t st, const double *LU, int n, const int *piv, const double *colsum, const int *status,
                    double *rcond);
// getrf with the dgecon estimate running on the context's side stream (forked after the factors,
// joined by lu_rcond_join); returns TTK_OK with *forked = 1, or the one-kernel path (*forked = 0)
int lu_factor_fork_rcond(hipStream_t st, double *A, int n, int *piv, double *work, int *forked);
int lu_rcond_join(hipStream_t st);
// getrs for nrhs columns of B (one workgroup per column, n <= 12000)
int lu_solve_cols(hipStream_t st, const double *LU, int n, const int *piv, double *B, int nrhs, int ldb);
// ttk_linalg.hip: ttk_qr of A given column-major (At, n x m row-major) returning Q^T (k x m
// row-major) and R as ttk_qr does, bit for bit; TTK_ERR_ARG, nothing launched, for shapes that
// take the blocked QR (the caller transposes and calls ttk_qr)
int qr_colmajor(void *stream, const double *At, int m, int n, double *Qt, double *R, double *work);

// ttk_contract.hip: grouped launches of independent offset-table GEMM problems (the einsum
// engine's batches).  gemm_groupable(): the problem runs on the plain 32x32-tile kernel when
// launched alone (no split-K, no 64x64 throughput variant), so a grouped launch computes every
// output element with the same operations in the same order (bit-identical).
struct GemmProblem {
  const double *A, *B;
  double *C;
  const int64_t *offs;
  int nb, M, N, K;
  double alpha, beta;
};
bool gemm_groupable(int nb, int M, int N, int K);
int gemm_group(hipStream_t st, const GemmProblem *p, int n);
// ttk_einsum.hip: launch the pending nodes of an open einsum batch (stream order for other launches)
int batch_barrier(void *stream);
// ttk_einsum.hip: one application of the current context's Schur operator handle on `stream`
int schur_apply(void *stream, int64_t handle, const double *v, double *out);
}  // namespace ttk

#endif
