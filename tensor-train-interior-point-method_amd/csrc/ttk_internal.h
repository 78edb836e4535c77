// Internal (non-ABI) entry points shared between libttk translation units.
#ifndef TTK_INTERNAL_H
#define TTK_INTERNAL_H

#include <hip/hip_runtime.h>

namespace ttk {
// ttk_dense.hip: blocked multi-workgroup Cholesky (status = LAPACK info, device int) and
// triangular solve op(L) X = B; both enqueue on `st` without synchronising.
int cholesky_blocked(hipStream_t st, double *A, int n, int *status);
int trsm_blocked(hipStream_t st, const double *L, int n, double *B, int nrhs, int ldb, int trans);
}  // namespace ttk

#endif
