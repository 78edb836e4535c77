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
  ttk::staged_copy<4>(kb * kb, tid, 256, [&](int e) { return A[(int64_t)(k0 + e / kb) * n + k0 + e % kb]; },
                      [&](int e, double v) { Ls[e / kb][e % kb] = v; });
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
  ttk::staged_copy<4>(kb * kb, tid, 256, [&](int e) { return A[(int64_t)(k0 + e / kb) * n + k0 + e % kb]; },
                      [&](int e, double v) { Ls[e / kb][e % kb] = v; });
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
  ttk::staged_copy<4>(
      kb * kb, tid, 256,
      [&](int e) {
        const int i = e / kb, j = e - i * kb;
        return trans ? L[(int64_t)(r0 + j) * n + r0 + i] : L[(int64_t)(r0 + i) * n + r0 + j];
      },
      [&](int e, double v) { Ls[e / kb][e % kb] = v; });
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


// ---------------------------------------------------------------- blocked LU (dgetrf) + gecon
// Per NB-column panel: (1) dgetf2 of the panel over rows [k0, n) in one workgroup (idamax pivot:
// first index of the largest |a|; rows swapped inside the panel only), (2) the panel's row swaps
// on every other column (dlaswp, one thread per column), (3) U12 = L11^-1 A12 (one thread per
// column, L11 in LDS), (4) A22 -= L21 U12 on fp64 MFMA.  LAPACK's right-looking dgetrf order.
// The 1-norm condition estimate (dgecon with dlacn2's Hager/Higham iteration) then runs in one
// workgroup on 32-row blocks: wave 0 solves the diagonal block with lane shuffles, all waves
// apply the block to the remaining rows, so a triangular solve costs n/16 barriers, not 2n.

__global__ __launch_bounds__(256) void colsum_kernel(const double *__restrict__ A, int n, double *__restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n) return;
  // the plain loop's additions in its order, the next 8 rows' loads in flight (one L2 round trip per 8
  // rows instead of per row: n = 1000 was ~0.25 ms on 4 workgroups)
  out[c] = ttk::sum_ahead<8>(n, [&](int r) { return fabs(A[(int64_t)r * n + c]); }, 0.0);
}

// row i of a panel step: l = a_ic / d, a_ij -= l u_j for j in (c, kb) -- `pi` (row i) and `prow` (the
// pivot row c < i) never overlap; saying so lets the u_j / a_ij loads issue ahead of the stores
// (with possible aliasing every element waited for the previous element's store: one LDS or L2
// round trip per element).  The same operations as the plain loop: bit-identical.
__device__ __forceinline__ void panel_row_update(double *__restrict__ pi, const double *__restrict__ prow, int c,
                                                 int kb, double inv) {
  const double l = pi[c] * inv;
  pi[c] = l;
#pragma unroll 8
  for (int cc = c + 1; cc < kb; ++cc) pi[cc] -= l * prow[cc];
}

__global__ __launch_bounds__(1024) void getf2_panel_kernel(double *A, int n, int k0, int kb, int *piv, int *status) {
  __shared__ double wv[16];
  __shared__ int wi[16];
  __shared__ int s_p;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int c = 0; c < kb; ++c) {
    const int j = k0 + c;
    double best = -1.0;
    int bi = j;
    for (int i = j + tid; i < n; i += 1024) {
      const double v = fabs(A[(int64_t)i * n + j]);
      if (v > best) {
        best = v;
        bi = i;
      }
    }
    ttk::wave_argmax(best, bi);  // DPP + readlane: the same winner as the shuffle butterfly
    if (lane == 0) {
      wv[wid] = best;
      wi[wid] = bi;
    }
    __syncthreads();
    if (tid == 0) {
      double b = wv[0];
      int p = wi[0];
      for (int w = 1; w < 16; ++w)
        if (wv[w] > b || (wv[w] == b && wi[w] < p)) {
          b = wv[w];
          p = wi[w];
        }
      s_p = p;
      piv[j] = p;
    }
    __syncthreads();
    const int p = s_p;
    if (p != j && tid < kb) {
      double *a = A + (int64_t)j * n + k0 + tid, *b = A + (int64_t)p * n + k0 + tid;
      const double t = *a;
      *a = *b;
      *b = t;
    }
    __syncthreads();
    const double d = A[(int64_t)j * n + j];
    if (d == 0.0) {  // LAPACK: info = first zero pivot, no scaling, factorisation continues
      if (tid == 0 && *status == 0) *status = j + 1;
      continue;
    }
    const double inv = 1.0 / d;
    const double *prow = A + (int64_t)j * n + k0;
    for (int i = j + 1 + tid; i < n; i += 1024) panel_row_update(A + (int64_t)i * n + k0, prow, c, kb, inv);
    __syncthreads();
  }
}

// the same panel factorisation with the (n-k0) x kb panel staged in LDS (row stride kb+1); any block
// size (a multiple of 64, <= 1024): lu_blocked launches one thread per panel row up to 1024, so a
// short panel synchronises fewer waves (the pivot is the same idamax winner whatever the layout)
__global__ __launch_bounds__(1024) void getf2_panel_lds_kernel(double *A, int n, int k0, int kb, int *piv,
                                                               int *status) {
  extern __shared__ double P[];
  __shared__ double wv[16];
  __shared__ int wi[16];
  __shared__ int s_p;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nt = blockDim.x, nw = nt >> 6;
  const int rows = n - k0, ld = kb + 1;
  ttk::staged_copy<8>(rows * kb, tid, nt, [&](int e) { return A[(int64_t)(k0 + e / kb) * n + k0 + e % kb]; },
                      [&](int e, double v) { P[(e / kb) * ld + e % kb] = v; });
  __syncthreads();
  for (int c = 0; c < kb; ++c) {
    double best = -1.0;
    int bi = c;
    for (int i = c + tid; i < rows; i += nt) {
      const double v = fabs(P[i * ld + c]);
      if (v > best) {
        best = v;
        bi = i;
      }
    }
    ttk::wave_argmax(best, bi);  // DPP + readlane: the same winner as the shuffle butterfly
    if (lane == 0) {
      wv[wid] = best;
      wi[wid] = bi;
    }
    __syncthreads();
    if (tid < 64) {  // wave 0: reduce the nw wave winners, swap the two panel rows
      double b = tid < nw ? wv[tid] : -2.0;
      int p = tid < nw ? wi[tid] : 0x7fffffff;
      ttk::wave_argmax(b, p);  // uniform over the wave
      if (p != c && tid < kb) {
        const double t = P[c * ld + tid];
        P[c * ld + tid] = P[p * ld + tid];
        P[p * ld + tid] = t;
      }
      if (tid == 0) {
        s_p = p;
        piv[k0 + c] = k0 + p;
      }
    }
    __syncthreads();
    const double d = P[c * ld + c];
    if (d == 0.0) {
      if (tid == 0 && *status == 0) *status = k0 + c + 1;
      continue;
    }
    const double inv = 1.0 / d;
    const double *prow = P + c * ld;
    for (int i = c + 1 + tid; i < rows; i += nt) panel_row_update(P + i * ld, prow, c, kb, inv);
    __syncthreads();
  }
  for (int e = tid; e < rows * kb; e += nt) {
    const int i = e / kb, c = e - i * kb;
    A[(int64_t)(k0 + i) * n + k0 + c] = P[i * ld + c];
  }
}

// The same panel factorisation with the panel in REGISTERS: thread t owns panel rows t, t + 1024, ...
// (R of them, KB columns each, kb <= KB used), so a column step touches memory only for the
// pivot search's 16 wave winners and the pivot row's broadcast -- two barriers per column, no
// global or LDS round trip per element (getf2_panel_kernel: a strided global scan and update per
// column; the LDS kernel: an LDS pass per column).  The same operations in the same order on every
// element (idamax winner, swap of the whole panel row, l = a * (1 / d), a -= l * u): bit-identical
// to both.  Double-buffered broadcast slots (column parity) leave the next column's writes behind
// the current column's second barrier.
// a copy the optimiser cannot look through (no instruction is emitted)
__device__ __forceinline__ double opaque(double x) {
  asm volatile("" : "+v"(x));
  return x;
}

template <int KB, int R>
struct PanelRegs {
  double r[R][KB];
  double (*cv)[16];
  int (*ci)[16];
  double (*prow_s)[KB];
  double (*crow_s)[KB];
  double *A;
  int n, k0, kb, rows, tid, lane, wid;
  int *piv, *status;

  // column C of the panel (C a template parameter: every r[][] index is compile-time)
  template <int C>
  __device__ __forceinline__ void column() {
    if constexpr (C < KB) {
      if (C < kb) {
        constexpr int b = C & 1;
        double best = -1.0;
        int bi = C;
#pragma unroll
        for (int q = 0; q < R; ++q) {
          const int i = tid + 1024 * q;
          if (i >= C && i < rows) {
            const double v = fabs(r[q][C]);
            if (v > best) {
              best = v;
              bi = i;
            }
          }
        }
        ttk::wave_argmax(best, bi);
        if (lane == 0) {
          cv[b][wid] = best;
          ci[b][wid] = bi;
        }
        __syncthreads();
        double pb = lane < 16 ? cv[b][lane] : -2.0;
        int p = lane < 16 ? ci[b][lane] : 0x7fffffff;
        ttk::wave_argmax(pb, p);  // every wave reduces the 16 winners itself: uniform p, no third barrier
        const int pt = p & 1023, pq = p >> 10;
        if (tid == pt) {  // row pq of this thread, picked by value selects behind an opaque copy (a
                          // select of two loads would fold into one load of a run-time index and
                          // send r[][] to scratch)
#pragma unroll
          for (int cc = 0; cc < KB; ++cc) {
            double v = opaque(r[0][cc]);
#pragma unroll
            for (int q = 1; q < R; ++q) v = q == pq ? opaque(r[q][cc]) : v;
            prow_s[b][cc] = v;
          }
        }
        if (p != C && tid == C) {
#pragma unroll
          for (int cc = 0; cc < KB; ++cc) crow_s[b][cc] = r[0][cc];
        }
        if (tid == 0) piv[k0 + C] = k0 + p;
        __syncthreads();
        if (p != C) {
          if (tid == C) {
#pragma unroll
            for (int cc = 0; cc < KB; ++cc) r[0][cc] = prow_s[b][cc];
          }
          if (tid == pt) {
#pragma unroll
            for (int cc = 0; cc < KB; ++cc) {
              const double v = crow_s[b][cc];
#pragma unroll
              for (int q = 0; q < R; ++q) r[q][cc] = q == pq ? v : opaque(r[q][cc]);
            }
          }
        }
        const double d = prow_s[b][C];
        if (d == 0.0) {  // LAPACK: info = first zero pivot, no scaling, factorisation continues
          if (tid == 0 && *status == 0) *status = k0 + C + 1;
        } else {
          const double inv = 1.0 / d;
#pragma unroll
          for (int q = 0; q < R; ++q) {
            const int i = tid + 1024 * q;
            if (i > C && i < rows) {
              const double l = r[q][C] * inv;
              r[q][C] = l;
#pragma unroll
              for (int cc = C + 1; cc < KB; ++cc)
                if (cc < kb) r[q][cc] -= l * prow_s[b][cc];
            }
          }
        }
      }
      column<C + 1>();
    }
  }
};

template <int KB, int R>
__global__ __launch_bounds__(1024) void getf2_panel_reg_kernel(double *A, int n, int k0, int kb, int *piv,
                                                               int *status) {
  __shared__ double cv[2][16];
  __shared__ int ci[2][16];
  __shared__ double prow_s[2][KB], crow_s[2][KB];
  PanelRegs<KB, R> P;
  P.cv = cv;
  P.ci = ci;
  P.prow_s = prow_s;
  P.crow_s = crow_s;
  P.A = A;
  P.n = n;
  P.k0 = k0;
  P.kb = kb;
  P.rows = n - k0;
  P.tid = threadIdx.x;
  P.lane = threadIdx.x & 63;
  P.wid = threadIdx.x >> 6;
  P.piv = piv;
  P.status = status;
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int i = P.tid + 1024 * q;
    const double *src = A + (int64_t)(k0 + i) * n + k0;
#pragma unroll
    for (int c = 0; c < KB; ++c) P.r[q][c] = (i < P.rows && c < kb) ? src[c] : 0.0;
  }
  P.template column<0>();
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int i = P.tid + 1024 * q;
    double *dst = A + (int64_t)(k0 + i) * n + k0;
    if (i < P.rows) {
#pragma unroll
      for (int c = 0; c < KB; ++c)
        if (c < kb) dst[c] = P.r[q][c];
    }
  }
}

// row swaps of panel [k0, k0+kb) on the columns outside it
__global__ __launch_bounds__(256) void laswp_kernel(double *A, int n, int k0, int kb, const int *piv) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n || (c >= k0 && c < k0 + kb)) return;
  for (int jj = k0; jj < k0 + kb; ++jj) {
    const int p = piv[jj];
    if (p != jj) {
      const double t = A[(int64_t)jj * n + c];
      A[(int64_t)jj * n + c] = A[(int64_t)p * n + c];
      A[(int64_t)p * n + c] = t;
    }
  }
}

// laswp_kernel and lu_u12_kernel in one launch: thread idx owns column c (every column outside the
// panel), applies the panel's row swaps to it, and -- right of the panel -- then solves its U12 column
// against L11 (staged in LDS; the panel columns are not swapped here, so L11 is final).  Per column
// the same operations as the two launches: bit-identical.
__global__ __launch_bounds__(256) void lu_swap_u12_kernel(double *A, int n, int k0, int kb, const int *piv) {
  __shared__ double Ls[NB][NB + 1];
  const int tid = threadIdx.x;
  const int idx = blockIdx.x * 256 + tid, c = idx < k0 ? idx : idx + kb;
  const bool right = (int)(blockIdx.x * 256 + 255) >= k0;  // the block has columns right of the panel
  if (right) {
    ttk::staged_copy<4>(kb * kb, tid, 256, [&](int e) { return A[(int64_t)(k0 + e / kb) * n + k0 + e % kb]; },
                        [&](int e, double v) { Ls[e / kb][e % kb] = v; });
    __syncthreads();
  }
  if (c >= n) return;
  for (int jj = k0; jj < k0 + kb; ++jj) {
    const int p = piv[jj];
    if (p != jj) {
      const double t = A[(int64_t)jj * n + c];
      A[(int64_t)jj * n + c] = A[(int64_t)p * n + c];
      A[(int64_t)p * n + c] = t;
    }
  }
  if (c < k0 + kb) return;
  double x[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) x[q] = q < kb ? A[(int64_t)(k0 + q) * n + c] : 0.0;
#pragma unroll
  for (int q = 1; q < NB; ++q) {
    if (q < kb) {
      double v = x[q];
#pragma unroll
      for (int p = 0; p < NB; ++p)
        if (p < q) v -= Ls[q][p] * x[p];
      x[q] = v;
    }
  }
#pragma unroll
  for (int q = 1; q < NB; ++q)
    if (q < kb) A[(int64_t)(k0 + q) * n + c] = x[q];
}

// U12 = L11^-1 A12 (L11 unit lower kb x kb), one thread per column c >= k0+kb
__global__ __launch_bounds__(256) void lu_u12_kernel(double *A, int n, int k0, int kb) {
  __shared__ double Ls[NB][NB + 1];
  const int tid = threadIdx.x;
  ttk::staged_copy<4>(kb * kb, tid, 256, [&](int e) { return A[(int64_t)(k0 + e / kb) * n + k0 + e % kb]; },
                      [&](int e, double v) { Ls[e / kb][e % kb] = v; });
  __syncthreads();
  const int c = k0 + kb + blockIdx.x * 256 + tid;
  if (c >= n) return;
  double x[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) x[q] = q < kb ? A[(int64_t)(k0 + q) * n + c] : 0.0;
#pragma unroll
  for (int q = 1; q < NB; ++q) {
    if (q < kb) {
      double v = x[q];
#pragma unroll
      for (int p = 0; p < NB; ++p)
        if (p < q) v -= Ls[q][p] * x[p];
      x[q] = v;
    }
  }
#pragma unroll
  for (int q = 1; q < NB; ++q)
    if (q < kb) A[(int64_t)(k0 + q) * n + c] = x[q];
}

constexpr int TB = 32;  // diagonal block of the one-workgroup triangular solves

// x[r] -= sum_p LU[r][b0+p] x[b0+p] for r in [r0, r1): half-waves own rows (32 lanes over the
// block's columns, coalesced); beyond 4096 rows one thread per row
__device__ __forceinline__ double row_dot(const double *__restrict__ a, const double *x, int bs);
__device__ __forceinline__ void rows_update(const double *__restrict__ LU, int n, double *x, int b0, int bs, int r0, int r1) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, half = lane >> 5, hl = lane & 31;
  if (r1 - r0 > 4096) {
#pragma unroll 1
    for (int r = r0 + tid; r < r1; r += 1024) x[r] -= row_dot(LU + (int64_t)r * n + b0, x + b0, bs);
    return;
  }
  // two rows per wave, 32 lanes each; a half-wave's next 4 rows are loaded before any is reduced
  const double xv = hl < bs ? x[b0 + hl] : 0.0;
  for (int r = r0 + 2 * wid + half; r < r1; r += 128) {
    double a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = (hl < bs && r + 32 * u < r1) ? LU[(int64_t)(r + 32 * u) * n + b0 + hl] : 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      double v = hl < bs ? a[u] * xv : 0.0;
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      if (hl == 0 && r + 32 * u < r1) x[r + 32 * u] -= v;
    }
  }
}

// sum_p a[p] x[p] over one row segment (bs <= TB), loads issued ahead of the FMAs
__device__ __forceinline__ double row_dot(const double *__restrict__ a, const double *x, int bs) {
  double s0 = 0.0, s1 = 0.0;
#pragma unroll 2
  for (int p = 0; p < TB; p += 2) {  // rows beyond 4096 only: kept small (the unrolled form spilled)
    const double v0 = p < bs ? a[p] : 0.0, v1 = p + 1 < bs ? a[p + 1] : 0.0;
    s0 = fma(v0, p < bs ? x[p] : 0.0, s0);
    s1 = fma(v1, p + 1 < bs ? x[p + 1] : 0.0, s1);
  }
  return s0 + s1;
}

// sum_p a[p * lda] x[p] in p order (bs <= TB); ABS: sum_p |a[p * lda]| x[p]
template <bool ABS = false>
__device__ __forceinline__ double col_dot(const double *__restrict__ a, int lda, const double *x, int bs) {
  double v = 0.0;
#pragma unroll 8
  for (int p = 0; p < bs; ++p) v += (ABS ? fabs(a[(int64_t)p * lda]) : a[(int64_t)p * lda]) * x[p];
  return v;
}

// one workgroup (1024 threads): x (in LDS) <- A^-1 x (trans = 0) or A^-T x (trans = 1), with the
// dgetrf factors LU (row-major n x n) and pivots (staged in LDS: the swap chain is serial)
// perm / tmp (LDS, optional): the composed row permutation of the pivots (x_P[i] = x[perm[i]]) and an
// n-double buffer, so the swaps become one parallel gather instead of the serial swap chain
// (TRANS a template parameter and the body inlined: as a called function with a runtime flag the
// unrolled blocks of both directions spilled ~600 bytes per lane to scratch)
// ABS (TRANS = 1 only): the same sweep on the comparison matrices, x <- M(L)^-T M(U)^-T x with M(T) =
// |diag T| - |offdiag T| (Higham, Accuracy and Stability, Thm 8.12): for x >= 0 every term is
// non-negative, and |A^-T| <= P M(L)^-T M(U)^-T entrywise, so max(x) for x = e bounds ||A^-1||_1
template <int TRANS, bool ABS = false>
__device__ __forceinline__ void lu_solve_blk(const double *__restrict__ LU, int n, const int *__restrict__ piv,
                                             double *x, const int *perm = nullptr, double *tmp = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int half = lane >> 5, hl = lane & 31;
  if (!TRANS) {
    if (perm) {
      for (int i = tid; i < n; i += blockDim.x) tmp[i] = x[perm[i]];
      __syncthreads();
      for (int i = tid; i < n; i += blockDim.x) x[i] = tmp[i];
    } else if (tid == 0)
      for (int i = 0; i < n; ++i) {
        const int p = piv[i];
        if (p != i) {
          const double t = x[i];
          x[i] = x[p];
          x[p] = t;
        }
      }
    __syncthreads();
    for (int b0 = 0; b0 < n; b0 += TB) {  // L y = P x, L unit lower
      const int bs = n - b0 < TB ? n - b0 : TB;
      if (wid == 0) {
        double lr[TB];
        const double *row = LU + (int64_t)(b0 + hl) * n + b0;
#pragma unroll
        for (int p = 0; p < TB; ++p) lr[p] = (p < hl && hl < bs) ? row[p] : 0.0;
        double xq = hl < bs ? x[b0 + hl] : 0.0;
#pragma unroll
        for (int p = 0; p < TB - 1; ++p) {
          const double xp = ttk::readlane_d(xq, p);  // p uniform: a scalar broadcast, no LDS trip
          xq -= lr[p] * xp;
        }
        if (half == 0 && hl < bs) x[b0 + hl] = xq;
      }
      __syncthreads();
      rows_update(LU, n, x, b0, bs, b0 + bs, n);
      __syncthreads();
    }
    for (int bend = n; bend > 0; bend -= TB) {  // U z = y
      const int b0 = bend - TB > 0 ? bend - TB : 0, bs = bend - b0;
      if (wid == 0) {
        double ur[TB];
        const double *row = LU + (int64_t)(b0 + hl) * n + b0;
#pragma unroll
        for (int p = 0; p < TB; ++p) ur[p] = (p > hl && p < bs && hl < bs) ? row[p] : 0.0;
        const double d = hl < bs ? row[hl] : 1.0;
        double xq = hl < bs ? x[b0 + hl] : 0.0;
#pragma unroll
        for (int p = TB - 1; p >= 0; --p) {
          if (p < bs) {
            if (hl == p) xq = xq / d;
            const double xp = ttk::readlane_d(xq, p);  // p uniform: a scalar broadcast, no LDS trip
            xq -= ur[p] * xp;
          }
        }
        if (half == 0 && hl < bs) x[b0 + hl] = xq;
      }
      __syncthreads();
      rows_update(LU, n, x, b0, bs, 0, b0);
      __syncthreads();
    }
  } else {
    const double sg = ABS ? -1.0 : 1.0;  // M(T) negates the off-diagonal magnitudes
    for (int b0 = 0; b0 < n; b0 += TB) {  // U^T y = b (lower, non-unit)
      const int bs = n - b0 < TB ? n - b0 : TB;
      if (wid == 0) {
        double uc[TB];
#pragma unroll
        for (int p = 0; p < TB; ++p) {
          const double u = (p < hl && hl < bs) ? LU[(int64_t)(b0 + p) * n + b0 + hl] : 0.0;
          uc[p] = ABS ? fabs(u) : u;
        }
        const double dd = hl < bs ? LU[(int64_t)(b0 + hl) * n + b0 + hl] : 1.0;
        const double d = ABS ? fabs(dd) : dd;
        double xq = hl < bs ? x[b0 + hl] : 0.0;
#pragma unroll
        for (int p = 0; p < TB; ++p) {
          if (p < bs) {
            if (hl == p) xq = xq / d;
            const double xp = ttk::readlane_d(xq, p);  // p uniform: a scalar broadcast, no LDS trip
            xq -= sg * uc[p] * xp;
          }
        }
        if (half == 0 && hl < bs) x[b0 + hl] = xq;
      }
      __syncthreads();
#pragma unroll 1
      for (int r = b0 + bs + tid; r < n; r += 1024)  // one thread per row, coalesced over r
        x[r] -= sg * col_dot<ABS>(LU + (int64_t)b0 * n + r, n, x + b0, bs);
      __syncthreads();
    }
    for (int bend = n; bend > 0; bend -= TB) {  // L^T z = y (upper, unit)
      const int b0 = bend - TB > 0 ? bend - TB : 0, bs = bend - b0;
      if (wid == 0) {
        double lc[TB];
#pragma unroll
        for (int p = 0; p < TB; ++p) {
          const double l = (p > hl && p < bs && hl < bs) ? LU[(int64_t)(b0 + p) * n + b0 + hl] : 0.0;
          lc[p] = ABS ? fabs(l) : l;
        }
        double xq = hl < bs ? x[b0 + hl] : 0.0;
#pragma unroll
        for (int p = TB - 1; p >= 0; --p) {
          const double xp = ttk::readlane_d(xq, p);  // p uniform: a scalar broadcast, no LDS trip
          xq -= sg * lc[p] * xp;
        }
        if (half == 0 && hl < bs) x[b0 + hl] = xq;
      }
      __syncthreads();
#pragma unroll 1
      for (int r = tid; r < b0; r += 1024) x[r] -= sg * col_dot<ABS>(LU + (int64_t)b0 * n + r, n, x + b0, bs);
      __syncthreads();
    }
    if (perm) {  // the swaps in reverse order = the inverse permutation
      for (int i = tid; i < n; i += blockDim.x) tmp[perm[i]] = x[i];
      __syncthreads();
      for (int i = tid; i < n; i += blockDim.x) x[i] = tmp[i];
    } else if (tid == 0)
      for (int i = n - 1; i >= 0; --i) {
        const int p = piv[i];
        if (p != i) {
          const double t = x[i];
          x[i] = x[p];
          x[p] = t;
        }
      }
    __syncthreads();
  }
}

// rcond above which the comparison-matrix bound settles dgecon's LinAlgWarning test (eps = 2.2e-16):
// a margin of ~450x over eps for the bound's own rounding
constexpr double RCOND_CERT = 1e-13;

// dgecon (1-norm) from the factors: colsum = column sums of |A| before factorisation
__global__ __launch_bounds__(1024) void lu_rcond_kernel(const double *__restrict__ LU, int n, const int *gpiv,
                                                        const double *__restrict__ colsum, const int *status,
                                                        double *rcond_out, int use_perm, int exact) {
  extern __shared__ double xl[];
  double *x = xl, *xs = xl + n, *tmp = use_perm ? xl + 2 * n : nullptr;
  int *piv = reinterpret_cast<int *>(xl + (use_perm ? 3 : 2) * n), *perm = use_perm ? piv + n : nullptr;
  for (int i = threadIdx.x; i < n; i += blockDim.x) piv[i] = gpiv[i];
  if (use_perm) {  // compose the pivot swaps once for the up to 11 solves below
    for (int i = threadIdx.x; i < n; i += blockDim.x) perm[i] = i;
    __syncthreads();
    if (threadIdx.x == 0)
      for (int i = 0; i < n; ++i) {
        const int p = piv[i];
        if (p != i) {
          const int t = perm[i];
          perm[i] = perm[p];
          perm[p] = t;
        }
      }
  }
  __shared__ double red[16];
  __shared__ double rv[1024];
  __shared__ int ri[1024];
  __shared__ double s_est, s_anorm;
  const int tid = threadIdx.x, nt = blockDim.x;
  if (*status) {
    if (tid == 0) *rcond_out = 0.0;
    return;
  }
  double cm = 0.0;
  for (int c = tid; c < n; c += nt) cm = fmax(cm, colsum[c]);
  rv[tid] = cm;
  __syncthreads();
  if (tid == 0) {
    double mx = 0.0;
    for (int i = 0; i < nt; ++i) mx = fmax(mx, rv[i]);
    s_anorm = mx;
    s_est = 0.0;
  }
  // certified shortcut: bound = max(M(L)^-T M(U)^-T e) >= ||A^-1||_1 (lu_solve_blk ABS), and dlacn2's
  // estimate never exceeds ||A^-1||_1, so 1 / (anorm * bound) is a lower bound of the rcond that
  // dgecon returns.  When it already exceeds RCOND_CERT (>> eps) the LinAlgWarning decision
  // (rcond < eps) is settled and the bound is reported instead of running the estimator.
  for (int i = tid; i < n; i += nt) x[i] = 1.0;
  __syncthreads();
  lu_solve_blk<1, true>(LU, n, piv, x, perm, tmp);
  double bmax = 0.0;
  for (int i = tid; i < n; i += nt) bmax = fmax(bmax, x[i]);
  rv[tid] = bmax;
  __syncthreads();
  if (tid == 0) {
    double mx = 0.0;
    for (int i = 0; i < nt; ++i) mx = fmax(mx, rv[i]);
    const double lb = (s_anorm > 0.0 && mx > 0.0 && mx < INFINITY) ? (1.0 / s_anorm) / mx : 0.0;
    s_est = (!exact && lb >= RCOND_CERT) ? lb : 0.0;
  }
  __syncthreads();
  if (s_est > 0.0) {
    if (tid == 0) *rcond_out = s_est;
    return;
  }
  __syncthreads();
  if (tid == 0) s_est = 0.0;
  for (int i = tid; i < n; i += nt) x[i] = 1.0 / n;
  __syncthreads();
  int jlast = -1;
  for (int iter = 0; iter < 5; ++iter) {
    lu_solve_blk<0>(LU, n, piv, x, perm, tmp);
    double s1 = 0.0;
    for (int i = tid; i < n; i += nt) s1 += fabs(x[i]);
    s1 = ttk::block_sum(s1, red);
    if (iter > 0 && s1 <= s_est) {
      __syncthreads();
      break;
    }
    __syncthreads();
    if (tid == 0) s_est = s1;
    for (int i = tid; i < n; i += nt) xs[i] = (x[i] >= 0.0) ? 1.0 : -1.0;
    __syncthreads();
    lu_solve_blk<1>(LU, n, piv, xs, perm, tmp);
    double best = -1.0;
    int bi = 0;
    for (int i = tid; i < n; i += nt)
      if (fabs(xs[i]) > best) {
        best = fabs(xs[i]);
        bi = i;
      }
    // first index of max |z|: wave shuffles, then wave 0 over the 16 wave winners
    ttk::wave_argmax(best, bi);  // DPP + readlane: the same winner as the shuffle butterfly
    if ((tid & 63) == 0) {
      rv[tid >> 6] = best;
      ri[tid >> 6] = bi;
    }
    __syncthreads();
    if (tid < 64) {
      double b = tid < (nt >> 6) ? rv[tid] : -2.0;
      int p = tid < (nt >> 6) ? ri[tid] : 0x7fffffff;
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) {
        const double ob = __shfl_xor(b, o, 64);
        const int op = __shfl_xor(p, o, 64);
        if (ob > b || (ob == b && op < p)) {
          b = ob;
          p = op;
        }
      }
      if (tid == 0) ri[32] = p;
    }
    __syncthreads();
    const int jn = ri[32];
    __syncthreads();
    if (jn == jlast) break;
    jlast = jn;
    for (int i = tid; i < n; i += nt) x[i] = (i == jn) ? 1.0 : 0.0;
    __syncthreads();
  }
  for (int i = tid; i < n; i += nt) x[i] = ((i & 1) ? -1.0 : 1.0) * (1.0 + (n > 1 ? (double)i / (n - 1) : 0.0));
  __syncthreads();
  lu_solve_blk<0>(LU, n, piv, x, perm, tmp);
  double s1 = 0.0;
  for (int i = tid; i < n; i += nt) s1 += fabs(x[i]);
  s1 = ttk::block_sum(s1, red);
  if (tid == 0) {
    const double temp = 2.0 * s1 / (3.0 * n);
    const double est = fmax(s_est, temp);
    *rcond_out = (s_anorm == 0.0 || est == 0.0) ? 0.0 : (1.0 / s_anorm) / est;
  }
}

// getrs for a few right-hand sides: one workgroup per column, x in LDS
__global__ __launch_bounds__(1024) void lu_solve_cols_kernel(const double *__restrict__ LU, int n, const int *gpiv,
                                                             double *B, int ldb) {
  extern __shared__ double xl[];
  const int c = blockIdx.x, tid = threadIdx.x;
  int *piv = reinterpret_cast<int *>(xl + n);
  for (int i = tid; i < n; i += 1024) piv[i] = gpiv[i];
  for (int i = tid; i < n; i += 1024) xl[i] = B[(int64_t)i * ldb + c];
  __syncthreads();
  lu_solve_blk<0>(LU, n, piv, xl);
  for (int i = tid; i < n; i += 1024) B[(int64_t)i * ldb + c] = xl[i];
}

}  // namespace

namespace ttk {

// TTK_LU_REG_PANEL=0: the panels on the LDS / global-memory kernels (bit-identical; diagnostics)
// TTK_LU_SWAP_U12=0: the row swaps and the U12 solve as two launches (bit-identical; diagnostics)
static const int g_lu_swap_u12 = getenv("TTK_LU_SWAP_U12") ? atoi(getenv("TTK_LU_SWAP_U12")) : 1;
// TTK_LU_PANEL_NARROW=0: the LDS panel kernel always at 1024 threads (bit-identical; diagnostics)
static const int g_lu_panel_narrow = getenv("TTK_LU_PANEL_NARROW") ? atoi(getenv("TTK_LU_PANEL_NARROW")) : 1;
static const int g_lu_reg_panel = getenv("TTK_LU_REG_PANEL") ? atoi(getenv("TTK_LU_REG_PANEL")) : 1;

int lu_blocked(hipStream_t st, double *A, int n, int *piv, double *work, int *status, double *rcond, int want_rcond) {
  TTK_HIP(hipMemsetAsync(status, 0, sizeof(int), st));
  double *colsum = work;  // n doubles
  if (want_rcond) hipLaunchKernelGGL(colsum_kernel, dim3((n + 255) / 256), dim3(256), 0, st, A, n, colsum);
  for (int k0 = 0; k0 < n;) {
    // widest panel (32, 16 or 8 columns) whose (n-k0) x kb block fits the 150 KB LDS staging
    int kb = NB;
    while (kb > 8 && (size_t)(n - k0) * (kb + 1) * sizeof(double) > 150000) kb >>= 1;
    if (kb > n - k0) kb = n - k0;
    const size_t pshm = (size_t)(n - k0) * (kb + 1) * sizeof(double);
    const int rq = (n - k0 + 1023) / 1024;  // panel rows per thread of the register kernel
    // panels that do not fit the LDS staging (kb = 8, more than 2083 rows) run in registers; where the
    // LDS kernel applies it is the faster one (tools/bench_lu.py: n = 1000 4.38 vs 4.66 ms with every
    // panel in registers; n = 3120 37.1 -> 24.0 ms, 3600 51.7 -> 31.6 ms with the global-memory panels
    // replaced)
    if (g_lu_reg_panel && pshm > 150000 && kb <= 8 && rq <= 4) {
      if (rq == 3)  // rows > 2083 (pshm > 150000): 3 or 4 rows per thread
        hipLaunchKernelGGL((getf2_panel_reg_kernel<8, 3>), dim3(1), dim3(1024), 0, st, A, n, k0, kb, piv, status);
      else
        hipLaunchKernelGGL((getf2_panel_reg_kernel<8, 4>), dim3(1), dim3(1024), 0, st, A, n, k0, kb, piv, status);
    } else if (pshm <= 150000) {
      if (pshm > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(getf2_panel_lds_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)pshm);
      const int ntp = g_lu_panel_narrow ? ((n - k0 + 63) / 64 * 64 < 1024 ? (n - k0 + 63) / 64 * 64 : 1024) : 1024;
      hipLaunchKernelGGL(getf2_panel_lds_kernel, dim3(1), dim3(ntp), pshm, st, A, n, k0, kb, piv, status);
    } else {
      hipLaunchKernelGGL(getf2_panel_kernel, dim3(1), dim3(1024), 0, st, A, n, k0, kb, piv, status);
    }
    const int rest = n - k0 - kb;
    if (g_lu_swap_u12) {
      if (n - kb > 0)
        hipLaunchKernelGGL(lu_swap_u12_kernel, dim3((n - kb + 255) / 256), dim3(256), 0, st, A, n, k0, kb, piv);
    } else {
      hipLaunchKernelGGL(laswp_kernel, dim3((n + 255) / 256), dim3(256), 0, st, A, n, k0, kb, piv);
      if (rest > 0)
        hipLaunchKernelGGL(lu_u12_kernel, dim3((rest + 255) / 256), dim3(256), 0, st, A, n, k0, kb);
    }
    if (rest > 0) {
      dim3 grid((rest + GT - 1) / GT, (rest + GT - 1) / GT);
      hipLaunchKernelGGL((gemm_strided_kernel<false, false>), grid, dim3(256), 0, st,
                         A + (int64_t)(k0 + kb) * n + k0, n, A + (int64_t)k0 * n + k0 + kb, n,
                         A + (int64_t)(k0 + kb) * n + k0 + kb, n, rest, rest, kb, -1.0, 1.0, 0);
    }
    TTK_LAUNCH_CHECK();
    k0 += kb;
  }
  if (want_rcond == 1) return lu_rcond_launch(st, A, n, piv, colsum, status, rcond);
  return TTK_OK;
}

int lu_rcond_launch(hipStream_t st, const double *LU, int n, const int *piv, const double *colsum, const int *status,
                    double *rcond) {
  // x, xs (+ the permutation buffer and perm when they fit next to the kernel's static LDS)
  const size_t shm_perm = 3 * (size_t)n * sizeof(double) + 2 * (size_t)n * sizeof(int);
  const int use_perm = shm_perm <= 140000;
  const size_t shm = use_perm ? shm_perm : 2 * (size_t)n * sizeof(double) + (size_t)n * sizeof(int);
  if (shm > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(lu_rcond_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  const int exact = ttk::ctx().knob[TTK_KNOB_RCOND_EXACT] != 0;
  hipLaunchKernelGGL(lu_rcond_kernel, dim3(1), dim3(1024), shm, st, LU, n, piv, colsum, status, rcond, use_perm,
                     exact);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int lu_solve_cols(hipStream_t st, const double *LU, int n, const int *piv, double *B, int nrhs, int ldb) {
  const size_t shm = (size_t)n * (sizeof(double) + sizeof(int));
  if (shm > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(lu_solve_cols_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL(lu_solve_cols_kernel, dim3(nrhs), dim3(1024), shm, st, LU, n, piv, B, ldb);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}


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
