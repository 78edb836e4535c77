// Blocked multi-workgroup Cholesky and triangular solves for the dense Schur local solves of the
// high-rank configs (`_ipm_local_solver(_ineq)`, src/tt_ipm.py:204-211,300-319; m = 4 r R up to
// ~1600 at graphm_3 r=2).  The one-workgroup unblocked kernels in ttk_linalg.hip stream the whole
// trailing matrix through one CU per column (O(n^3) element updates at one CU's L2 bandwidth);
// here each NB-column panel costs three launches over the chip:
//   Cholesky  (1) potf2 of the NB x NB diagonal block in LDS (one workgroup, status on failure)
//             (2) L21 = A21 L11^-T, rows in parallel, L11 in LDS
//             (3) A22 -= L21 L21^T on fp64 MFMA, lower tiles only
//   TRSM      (1) the NB-row diagonal block solve, one thread per RHS column, L block in LDS
//             (2) rest -= L(rest, blk) X(blk) on fp64 MFMA
// Same arithmetic as LAPACK's blocked dpotrf/dtrsm (right-looking), so results agree with the
// unblocked kernels to rounding.  Row-major storage, leading dimension = n (L) / ldb (B).
#include <hip/hip_runtime.h>

#include "ttk_common.h"
#include "ttk_internal.h"

namespace {

constexpr int NB = 32;                // panel width
constexpr int GT = 32, GK = 16;       // GEMM tile (32 x 32 outputs, K stages of 16)

typedef double double4_t __attribute__((ext_vector_type(4)));

// C(i,j) = beta C(i,j) + alpha sum_k A(i,k) B(k,j) on rows [0,M) x cols [0,N), K terms.
// A(i,k) = TA ? A[k*lda+i] : A[i*lda+k];  B(k,j) = TB ? B[j*ldb+k] : B[k*ldb+j].
// lower_only: skip tiles strictly above the diagonal (symmetric rank-k update).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_strided_kernel(const double *__restrict__ A, int lda,
                                                           const double *__restrict__ B, int ldb,
                                                           double *__restrict__ C, int ldc, int M, int N, int K,
                                                           double alpha, double beta, int lower_only) {
  const int n0 = blockIdx.x * GT, m0 = blockIdx.y * GT;
  if (lower_only && n0 > m0 + GT - 1) return;
  __shared__ double As[GK][GT + 1];
  __shared__ double Bs[GK][GT + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int l_mn = tid & 31, l_k = tid >> 5;
  const bool am = m0 + l_mn < M, bn = n0 + l_mn < N;
  auto ld_a = [&](int k) -> double {
    if (!am || k >= K) return 0.0;
    const int i = m0 + l_mn;
    return TA ? A[(int64_t)k * lda + i] : A[(int64_t)i * lda + k];
  };
  auto ld_b = [&](int k) -> double {
    if (!bn || k >= K) return 0.0;
    const int j = n0 + l_mn;
    return TB ? B[(int64_t)j * ldb + k] : B[(int64_t)k * ldb + j];
  };
  double ra0 = ld_a(l_k), ra1 = ld_a(l_k + 8), rb0 = ld_b(l_k), rb1 = ld_b(l_k + 8);
  double4_t acc = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < K; k0 += GK) {
    As[l_k][l_mn] = ra0;
    As[l_k + 8][l_mn] = ra1;
    Bs[l_k][l_mn] = rb0;
    Bs[l_k + 8][l_mn] = rb1;
    __syncthreads();
    if (k0 + GK < K) {
      ra0 = ld_a(k0 + GK + l_k);
      ra1 = ld_a(k0 + GK + l_k + 8);
      rb0 = ld_b(k0 + GK + l_k);
      rb1 = ld_b(k0 + GK + l_k + 8);
    }
#pragma unroll
    for (int s = 0; s < GK / 4; ++s) {
      const double a = As[s * 4 + (lane >> 4)][wr * 16 + (lane & 15)];
      const double b = Bs[s * 4 + (lane >> 4)][wc * 16 + (lane & 15)];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int col = n0 + wc * 16 + (lane & 15);
  if (col >= N) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m0 + wr * 16 + (lane >> 4) + 4 * r;
    if (row < M) {
      double *p = C + (int64_t)row * ldc + col;
      *p = beta * (*p) + alpha * acc[r];
    }
  }
}

// unblocked Cholesky of the kb x kb diagonal block at A + k0*(n+1), in LDS; status = first failing
// global column + 1 (LAPACK info), left untouched on success
__global__ __launch_bounds__(256) void potf2_block_kernel(double *A, int n, int k0, int kb, int *status) {
  __shared__ double Ls[NB][NB + 1];
  __shared__ int s_fail;
  const int tid = threadIdx.x;
  if (*status) return;  // an earlier panel failed: LAPACK stops there
  for (int e = tid; e < kb * kb; e += 256) {
    const int i = e / kb, j = e - i * kb;
    Ls[i][j] = A[(int64_t)(k0 + i) * n + k0 + j];
  }
  if (tid == 0) s_fail = 0;
  __syncthreads();
  for (int j = 0; j < kb; ++j) {
    if (tid == 0) {
      const double d = Ls[j][j];
      if (!(d > 0.0)) {
        s_fail = k0 + j + 1;
      } else {
        Ls[j][j] = sqrt(d);
      }
    }
    __syncthreads();
    if (s_fail) break;
    const double inv = 1.0 / Ls[j][j];
    for (int i = j + 1 + tid; i < kb; i += 256) Ls[i][j] *= inv;
    __syncthreads();
    const int t = kb - j - 1;
    for (int e = tid; e < t * t; e += 256) {
      const int i = j + 1 + e / t, c = j + 1 + e % t;
      if (c <= i) Ls[i][c] -= Ls[i][j] * Ls[c][j];
    }
    __syncthreads();
  }
  if (s_fail) {
    if (tid == 0) *status = s_fail;
    return;
  }
  for (int e = tid; e < kb * kb; e += 256) {
    const int i = e / kb, j = e - i * kb;
    if (j <= i) A[(int64_t)(k0 + i) * n + k0 + j] = Ls[i][j];
  }
}

// rows r >= k0+kb of the panel: x L11^T = a  (forward substitution over kb columns)
__global__ __launch_bounds__(256) void panel_trsm_kernel(double *A, int n, int k0, int kb, const int *status) {
  __shared__ double Ls[NB][NB + 1];
  if (*status) return;
  const int tid = threadIdx.x;
  for (int e = tid; e < kb * kb; e += 256) {
    const int i = e / kb, j = e - i * kb;
    Ls[i][j] = A[(int64_t)(k0 + i) * n + k0 + j];
  }
  __syncthreads();
  const int r = k0 + kb + blockIdx.x * 256 + tid;
  if (r >= n) return;
  double *a = A + (int64_t)r * n + k0;
  double x[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) x[j] = j < kb ? a[j] : 0.0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if (j < kb) {
      double s = x[j];
#pragma unroll
      for (int c = 0; c < NB; ++c)
        if (c < j) s -= x[c] * Ls[j][c];
      x[j] = s / Ls[j][j];
    }
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (j < kb) a[j] = x[j];
}

__global__ __launch_bounds__(256) void zero_upper_kernel(double *A, int n, const int *status) {
  if (*status) return;
  const int64_t e = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int i = (int)(e / n), c = (int)(e % n);
  if (c > i) A[e] = 0.0;
}

// diagonal-block solve of op(L) X = B for rows [r0, r0+kb): one thread per RHS column
__global__ __launch_bounds__(256) void trsm_diag_kernel(const double *__restrict__ L, int n, double *B, int nrhs,
                                                        int ldb, int r0, int kb, int trans) {
  __shared__ double Ls[NB][NB + 1];
  const int tid = threadIdx.x;
  for (int e = tid; e < kb * kb; e += 256) {
    const int i = e / kb, j = e - i * kb;
    Ls[i][j] = trans ? L[(int64_t)(r0 + j) * n + r0 + i] : L[(int64_t)(r0 + i) * n + r0 + j];
  }
  __syncthreads();
  const int c = blockIdx.x * 256 + tid;
  if (c >= nrhs) return;
  double x[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) x[j] = j < kb ? B[(int64_t)(r0 + j) * ldb + c] : 0.0;
  if (!trans) {  // forward: rows r0 .. r0+kb-1 ; Ls = L block (lower)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (j < kb) {
        double s = x[j];
#pragma unroll
        for (int q = 0; q < NB; ++q)
          if (q < j) s -= Ls[j][q] * x[q];
        x[j] = s / Ls[j][j];
      }
    }
  } else {  // backward with L^T: Ls[i][j] = L(r0+j, r0+i) is upper triangular
#pragma unroll
    for (int jj = NB - 1; jj >= 0; --jj) {
      if (jj < kb) {
        double s = x[jj];
#pragma unroll
        for (int q = 0; q < NB; ++q)
          if (q > jj && q < kb) s -= Ls[jj][q] * x[q];
        x[jj] = s / Ls[jj][jj];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (j < kb) B[(int64_t)(r0 + j) * ldb + c] = x[j];
}

}  // namespace

namespace ttk {

int cholesky_blocked(hipStream_t st, double *A, int n, int *status) {
  TTK_HIP(hipMemsetAsync(status, 0, sizeof(int), st));
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int kb = n - k0 < NB ? n - k0 : NB;
    hipLaunchKernelGGL(potf2_block_kernel, dim3(1), dim3(256), 0, st, A, n, k0, kb, status);
    const int rest = n - k0 - kb;
    if (rest > 0) {
      hipLaunchKernelGGL(panel_trsm_kernel, dim3((rest + 255) / 256), dim3(256), 0, st, A, n, k0, kb, status);
      // A22 -= L21 L21^T (lower tiles); L21 = A[k0+kb:, k0:k0+kb]
      double *L21 = A + (int64_t)(k0 + kb) * n + k0;
      double *A22 = A + (int64_t)(k0 + kb) * n + k0 + kb;
      dim3 grid((rest + GT - 1) / GT, (rest + GT - 1) / GT);
      hipLaunchKernelGGL((gemm_strided_kernel<false, true>), grid, dim3(256), 0, st, L21, n, L21, n, A22, n, rest,
                         rest, kb, -1.0, 1.0, 1);
    }
    TTK_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(zero_upper_kernel, dim3((unsigned)(((int64_t)n * n + 255) / 256)), dim3(256), 0, st, A, n,
                     status);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int trsm_blocked(hipStream_t st, const double *L, int n, double *B, int nrhs, int ldb, int trans) {
  for (int s = 0; s < n; s += NB) {
    const int kb = n - s < NB ? n - s : NB;
    // forward: block rows [s, s+kb); backward (L^T): block rows [n-s-kb, n-s)
    const int r0 = trans ? n - s - kb : s;
    hipLaunchKernelGGL(trsm_diag_kernel, dim3((nrhs + 255) / 256), dim3(256), 0, st, L, n, B, nrhs, ldb, r0, kb,
                       trans);
    const int rest = n - s - kb;
    if (rest > 0) {
      dim3 grid((nrhs + GT - 1) / GT, (rest + GT - 1) / GT);
      if (!trans) {  // B[r0+kb:, :] -= L[r0+kb:, r0:r0+kb] X[r0:r0+kb, :]
        hipLaunchKernelGGL((gemm_strided_kernel<false, false>), grid, dim3(256), 0, st,
                           L + (int64_t)(r0 + kb) * n + r0, n, B + (int64_t)r0 * ldb, ldb,
                           B + (int64_t)(r0 + kb) * ldb, ldb, rest, nrhs, kb, -1.0, 1.0, 0);
      } else {  // B[0:r0, :] -= L[r0:r0+kb, 0:r0]^T X[r0:r0+kb, :]
        hipLaunchKernelGGL((gemm_strided_kernel<true, false>), grid, dim3(256), 0, st, L + (int64_t)r0 * n, n,
                           B + (int64_t)r0 * ldb, ldb, B, ldb, rest, nrhs, kb, -1.0, 1.0, 0);
      }
    }
    TTK_LAUNCH_CHECK();
  }
  return TTK_OK;
}

}  // namespace ttk
