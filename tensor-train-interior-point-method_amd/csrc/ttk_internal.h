// Internal (non-ABI) entry points shared between libttk translation units.
#ifndef TTK_INTERNAL_H
#define TTK_INTERNAL_H

#include <hip/hip_runtime.h>

namespace ttk {
// ttk_dense.hip: blocked multi-workgroup Cholesky (status = LAPACK info, device int) and
// triangular solve op(L) X = B; both enqueue on `st` without synchronising.
int cholesky_blocked(hipStream_t st, double *A, int n, int *status);
int trsm_blocked(hipStream_t st, const double *L, int n, double *B, int nrhs, int ldb, int trans);
// blocked getrf (device pivots and LAPACK info in `status`) and, if want_rcond, the dgecon
// 1-norm estimate into device `rcond`; work >= n doubles.  Enqueued without synchronising.
int lu_blocked(hipStream_t st, double *A, int n, int *piv, double *work, int *status, double *rcond, int want_rcond);
// getrs for nrhs columns of B (one workgroup per column, n <= 12000)
int lu_solve_cols(hipStream_t st, const double *LU, int n, const int *piv, double *B, int nrhs, int ldb);

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
}  // namespace ttk

#endif
