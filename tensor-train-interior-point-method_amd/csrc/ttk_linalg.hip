// Small dense factorisations for the TT-IPM hot path, one workgroup per matrix.
//
// The matrices on the path are tiny (TT unfoldings <= ~200 x 200, local KKT blocks m <= ~500 at
// the BASELINE sizes), so each factorisation runs inside ONE workgroup: the working copy lives
// in LDS when it fits in 64 KiB and in an L2-resident global scratch otherwise (same code, flat
// pointers).  Latency, not FLOPs, bounds these kernels: one launch per factorisation replaces
// the reference's Python->SciPy->LAPACK round trip per call.
//
//  svd   : one-sided (Hestenes) Jacobi, round-robin parallel pair ordering, one wave per pair.
//          High relative accuracy in the singular values (the truncation rule
//          `prune_singular_vals`, cy_src/tt_ops_cy.pyx:161-177, reads them on the host).
//  qr    : Householder (LAPACK geqrf/orgqr sign convention beta = -sign(alpha)*||x||).
//  chol  : right-looking unblocked Cholesky, LAPACK potrf failure rule (d <= 0 or NaN).
//  trsm  : column-blocked forward / backward substitution, many workgroups over RHS columns.
//  lu    : getrf with partial pivoting (first max, like idamax) + gecon-style 1-norm rcond
//          estimate (Hager / Higham) for scipy.linalg.solve's ill-conditioning warning.
//  syev  : cyclic two-sided Jacobi with round-robin ordering (eigenvalues ascending).
#include <math.h>

#include "ttk_common.h"

namespace {

constexpr double EPS = 2.220446049250313e-16;
constexpr int LDS_DOUBLES = 20000;  // 160000 B of dynamic LDS (gfx950: 160 KiB per workgroup)

// round-robin (circle method) pair k of round r over P (even) items
__device__ __forceinline__ void rr_pair(int P, int r, int k, int &p, int &q) {
  if (k == 0) {
    p = r;
    q = P - 1;
  } else {
    p = (r + k) % (P - 1);
    q = (r - k + P - 1) % (P - 1);
  }
  if (p > q) {
    int t = p;
    p = q;
    q = t;
  }
}

// ------------------------------------------------------------------------------ SVD
// W: q x p column-major (column j at W + j*q), V: p x p column-major.
__global__ __launch_bounds__(1024) void svd_kernel(const double *__restrict__ A, int m, int n,
                                                   double *__restrict__ U, double *__restrict__ S,
                                                   double *__restrict__ Vt, double *__restrict__ gwork,
                                                   int use_lds) {
  extern __shared__ double lds[];
  __shared__ int any_rot;
  __shared__ double red[16];
  const bool tall = m >= n;
  const int p = tall ? n : m;  // columns to orthogonalise
  const int q = tall ? m : n;  // column length
  double *base = use_lds ? lds : gwork;
  double *W = base;
  double *V = W + (int64_t)q * p;
  double *sig = V + (int64_t)p * p;
  int *rank = reinterpret_cast<int *>(sig + p);
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  for (int64_t e = tid; e < (int64_t)q * p; e += nt) {
    const int j = (int)(e / q), i = (int)(e % q);
    W[e] = tall ? A[(int64_t)i * n + j] : A[(int64_t)j * n + i];
  }
  for (int64_t e = tid; e < (int64_t)p * p; e += nt) V[e] = ((e / p) == (e % p)) ? 1.0 : 0.0;
  __syncthreads();
  const int P = (p % 2) ? p + 1 : p;
  // rotate only when the columns are not orthogonal to working precision (LAPACK gesvj uses
  // sqrt(m)*eps; q*eps is the safe side that still converges quadratically)
  const double tol = EPS * (q > 16 ? (double)q : 16.0);
  for (int sweep = 0; sweep < 40; ++sweep) {
    if (tid == 0) any_rot = 0;
    __syncthreads();
    for (int r = 0; r < P - 1; ++r) {
      for (int k = wid; k < P / 2; k += nw) {
        int a, b;
        rr_pair(P, r, k, a, b);
        if (b >= p) continue;  // dummy partner
        double *wa = W + (int64_t)a * q, *wb = W + (int64_t)b * q;
        double al = 0.0, be = 0.0, ga = 0.0;
        for (int i = lane; i < q; i += 64) {
          const double x = wa[i], y = wb[i];
          al += x * x;
          be += y * y;
          ga += x * y;
        }
        al = ttk::wave_sum(al);
        be = ttk::wave_sum(be);
        ga = ttk::wave_sum(ga);
        if (al < 1e-300 || be < 1e-300) continue;
        if (fabs(ga) <= tol * sqrt(al) * sqrt(be)) continue;
        const double zeta = (be - al) / (2.0 * ga);
        double t;
        if (fabs(zeta) > 1e150)
          t = 0.5 / zeta;
        else
          t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
        for (int i = lane; i < q; i += 64) {
          const double x = wa[i], y = wb[i];
          wa[i] = c * x - s * y;
          wb[i] = s * x + c * y;
        }
        double *va = V + (int64_t)a * p, *vb = V + (int64_t)b * p;
        for (int i = lane; i < p; i += 64) {
          const double x = va[i], y = vb[i];
          va[i] = c * x - s * y;
          vb[i] = s * x + c * y;
        }
        if (lane == 0) any_rot = 1;
      }
      __syncthreads();
    }
    if (!any_rot) break;
    __syncthreads();
  }
  // singular values = column norms
  for (int j = wid; j < p; j += nw) {
    const double *wj = W + (int64_t)j * q;
    double s2 = 0.0;
    for (int i = lane; i < q; i += 64) s2 += wj[i] * wj[i];
    s2 = ttk::wave_sum(s2);
    if (lane == 0) sig[j] = sqrt(s2);
  }
  __syncthreads();
  for (int j = tid; j < p; j += nt) {
    int rk = 0;
    const double sj = sig[j];
    for (int i = 0; i < p; ++i) {
      const double si = sig[i];
      rk += (si > sj) || (si == sj && i < j);
    }
    rank[j] = rk;
  }
  __syncthreads();
  // left vectors: normalise columns (zero columns completed below)
  for (int j = wid; j < p; j += nw) {
    double *wj = W + (int64_t)j * q;
    const double sj = sig[j];
    if (sj > 0.0) {
      const double inv = 1.0 / sj;
      for (int i = lane; i < q; i += 64) wj[i] *= inv;
    }
  }
  __syncthreads();
  // complete zero-singular-value columns to an orthonormal set (rare; serial is fine)
  for (int j = 0; j < p; ++j) {
    if (sig[j] > 0.0) continue;
    double *wj = W + (int64_t)j * q;
    for (int cand = 0; cand < q; ++cand) {
      for (int i = tid; i < q; i += nt) wj[i] = (i == cand) ? 1.0 : 0.0;
      __syncthreads();
      for (int o = 0; o < p; ++o) {  // MGS against all other (already unit or completed) columns
        if (o == j || (sig[o] == 0.0 && o > j)) continue;
        const double *wo = W + (int64_t)o * q;
        double d = 0.0;
        for (int i = tid; i < q; i += nt) d += wo[i] * wj[i];
        d = ttk::block_sum(d, red);
        for (int i = tid; i < q; i += nt) wj[i] -= d * wo[i];
        __syncthreads();
      }
      double nn = 0.0;
      for (int i = tid; i < q; i += nt) nn += wj[i] * wj[i];
      nn = ttk::block_sum(nn, red);
      if (nn > 0.25) {
        const double inv = 1.0 / sqrt(nn);
        for (int i = tid; i < q; i += nt) wj[i] *= inv;
        __syncthreads();
        break;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  // write outputs: A = U diag(S) Vt, U (m x p), Vt (p x n)
  for (int j = tid; j < p; j += nt) S[rank[j]] = sig[j];
  if (tall) {
    for (int64_t e = tid; e < (int64_t)m * p; e += nt) {
      const int i = (int)(e / p), j = (int)(e % p);
      U[(int64_t)i * p + rank[j]] = W[(int64_t)j * q + i];
    }
    for (int64_t e = tid; e < (int64_t)p * n; e += nt) {
      const int j = (int)(e / n), i = (int)(e % n);
      Vt[(int64_t)rank[j] * n + i] = V[(int64_t)j * p + i];
    }
  } else {
    for (int64_t e = tid; e < (int64_t)m * p; e += nt) {
      const int i = (int)(e / p), j = (int)(e % p);
      U[(int64_t)i * p + rank[j]] = V[(int64_t)j * p + i];
    }
    for (int64_t e = tid; e < (int64_t)p * n; e += nt) {
      const int j = (int)(e / n), i = (int)(e % n);
      Vt[(int64_t)rank[j] * n + i] = W[(int64_t)j * q + i];
    }
  }
}

// ------------------------------------------------------------------------------ QR
// W: m x n column-major working copy; tau: k.
__global__ __launch_bounds__(1024) void qr_kernel(const double *__restrict__ A, int m, int n,
                                                  double *__restrict__ Q, double *__restrict__ R,
                                                  double *__restrict__ gwork, int use_lds) {
  extern __shared__ double lds[];
  __shared__ double red[16];
  __shared__ double s_beta, s_tau, s_scale;
  const int k = m < n ? m : n;
  double *W = use_lds ? lds : gwork;
  double *tau = W + (int64_t)m * n;
  double *Qc = tau + k;  // m x k column-major accumulation
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  for (int64_t e = tid; e < (int64_t)m * n; e += nt) {
    const int j = (int)(e / m), i = (int)(e % m);
    W[e] = A[(int64_t)i * n + j];
  }
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    double *wj = W + (int64_t)j * m;
    double s2 = 0.0;
    for (int i = j + 1 + tid; i < m; i += nt) s2 += wj[i] * wj[i];
    s2 = ttk::block_sum(s2, red);
    if (tid == 0) {
      const double alpha = wj[j];
      if (s2 == 0.0) {
        s_tau = 0.0;
        s_beta = alpha;
        s_scale = 0.0;
      } else {
        const double nrm = sqrt(alpha * alpha + s2);
        const double beta = (alpha >= 0.0) ? -nrm : nrm;
        s_tau = (beta - alpha) / beta;
        s_scale = 1.0 / (alpha - beta);
        s_beta = beta;
      }
    }
    __syncthreads();
    const double tj = s_tau, sc = s_scale;
    for (int i = j + 1 + tid; i < m; i += nt) wj[i] *= sc;
    __syncthreads();
    if (tid == 0) {
      wj[j] = s_beta;
      tau[j] = tj;
    }
    // apply H_j = I - tau v v^T (v = [1; wj[j+1:]]) to columns c > j, one wave per column
    if (tj != 0.0) {
      for (int c = j + 1 + wid; c < n; c += nw) {
        double *wc = W + (int64_t)c * m;
        double d = (lane == 0) ? wc[j] : 0.0;
        for (int i = j + 1 + lane; i < m; i += 64) d += wj[i] * wc[i];
        d = ttk::wave_sum(d) * tj;
        if (lane == 0) wc[j] -= d;
        for (int i = j + 1 + lane; i < m; i += 64) wc[i] -= d * wj[i];
      }
    }
    __syncthreads();
  }
  // R (k x n) row-major upper trapezoid
  for (int64_t e = tid; e < (int64_t)k * n; e += nt) {
    const int i = (int)(e / n), c = (int)(e % n);
    R[e] = (c >= i) ? W[(int64_t)c * m + i] : 0.0;
  }
  // Q = H_0 ... H_{k-1} [I_k; 0]
  for (int64_t e = tid; e < (int64_t)m * k; e += nt) {
    const int c = (int)(e / m), i = (int)(e % m);
    Qc[e] = (i == c) ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int j = k - 1; j >= 0; --j) {
    const double tj = tau[j];
    if (tj == 0.0) continue;
    const double *v = W + (int64_t)j * m;
    for (int c = j + wid; c < k; c += nw) {
      double *qc = Qc + (int64_t)c * m;
      double d = (lane == 0) ? qc[j] : 0.0;
      for (int i = j + 1 + lane; i < m; i += 64) d += v[i] * qc[i];
      d = ttk::wave_sum(d) * tj;
      if (lane == 0) qc[j] -= d;
      for (int i = j + 1 + lane; i < m; i += 64) qc[i] -= d * v[i];
    }
    __syncthreads();
  }
  for (int64_t e = tid; e < (int64_t)m * k; e += nt) {
    const int i = (int)(e / k), c = (int)(e % k);
    Q[e] = Qc[(int64_t)c * m + i];
  }
}

// ------------------------------------------------------------------------------ Cholesky
__global__ __launch_bounds__(1024) void chol_kernel(double *A, int n, int *status) {
  __shared__ double s_l;
  __shared__ int s_fail;
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) s_fail = 0;
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    if (tid == 0) {
      const double d = A[(int64_t)j * n + j];
      if (!(d > 0.0)) {
        s_fail = j + 1;
      } else {
        s_l = sqrt(d);
        A[(int64_t)j * n + j] = s_l;
      }
    }
    __syncthreads();
    if (s_fail) break;
    const double inv = 1.0 / s_l;
    for (int i = j + 1 + tid; i < n; i += nt) A[(int64_t)i * n + j] *= inv;
    __syncthreads();
    const int t = n - j - 1;
    for (int64_t e = tid; e < (int64_t)t * t; e += nt) {
      const int i = j + 1 + (int)(e / t), c = j + 1 + (int)(e % t);
      if (c <= i) A[(int64_t)i * n + c] -= A[(int64_t)i * n + j] * A[(int64_t)c * n + j];
    }
    __syncthreads();
  }
  if (!s_fail) {
    for (int64_t e = tid; e < (int64_t)n * n; e += nt) {
      const int i = (int)(e / n), c = (int)(e % n);
      if (c > i) A[e] = 0.0;
    }
  }
  if (tid == 0) *status = s_fail;
}

// ------------------------------------------------------------------------------ TRSM
// Solve op(L) X = B in place; L lower (n x n row-major); B (n x nrhs), leading dim ldb.
// Each workgroup owns 64 RHS columns; rows processed in order with right-looking updates.
__global__ __launch_bounds__(256) void trsm_kernel(const double *__restrict__ L, int n, double *B,
                                                   int nrhs, int ldb, int trans) {
  const int c0 = blockIdx.x * 64;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int ncol = min(64, nrhs - c0);
  if (ncol <= 0) return;
  for (int step = 0; step < n; ++step) {
    const int i = trans ? (n - 1 - step) : step;
    const double dinv = 1.0 / L[(int64_t)i * n + i];
    for (int c = tid; c < ncol; c += nt) B[(int64_t)i * ldb + c0 + c] *= dinv;
    __syncthreads();
    // update remaining rows
    const int rem = n - step - 1;
    for (int64_t e = tid; e < (int64_t)rem * ncol; e += nt) {
      const int rr = (int)(e / ncol), c = (int)(e % ncol);
      const int row = trans ? (i - 1 - rr) : (i + 1 + rr);
      const double lv = trans ? L[(int64_t)i * n + row] : L[(int64_t)row * n + i];
      B[(int64_t)row * ldb + c0 + c] -= lv * B[(int64_t)i * ldb + c0 + c];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------ LU (+ rcond)
// triangular solves with a single RHS vector in `x` using the packed LU (unit lower L, upper U)
__device__ void lu_vec_solve(const double *LU, int n, const int *piv, double *x, int trans) {
  const int tid = threadIdx.x, nt = blockDim.x;
  if (!trans) {
    // P x
    if (tid == 0)
      for (int i = 0; i < n; ++i) {
        const int p = piv[i];
        if (p != i) {
          const double t = x[i];
          x[i] = x[p];
          x[p] = t;
        }
      }
    __syncthreads();
    for (int i = 0; i < n; ++i) {  // L y = x (unit)
      const double xi = x[i];
      for (int r = i + 1 + tid; r < n; r += nt) x[r] -= LU[(int64_t)r * n + i] * xi;
      __syncthreads();
    }
    for (int i = n - 1; i >= 0; --i) {  // U z = y
      if (tid == 0) x[i] /= LU[(int64_t)i * n + i];
      __syncthreads();
      const double xi = x[i];
      for (int r = tid; r < i; r += nt) x[r] -= LU[(int64_t)r * n + i] * xi;
      __syncthreads();
    }
  } else {
    // A^T x = b: U^T y = b, L^T z = y, x = P^T z
    for (int i = 0; i < n; ++i) {
      if (tid == 0) x[i] /= LU[(int64_t)i * n + i];
      __syncthreads();
      const double xi = x[i];
      for (int r = i + 1 + tid; r < n; r += nt) x[r] -= LU[(int64_t)i * n + r] * xi;
      __syncthreads();
    }
    for (int i = n - 1; i >= 0; --i) {
      const double xi = x[i];
      for (int r = tid; r < i; r += nt) x[r] -= LU[(int64_t)i * n + r] * xi;
      __syncthreads();
    }
    if (tid == 0)
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

__global__ __launch_bounds__(1024) void lu_kernel(double *A, int n, int *piv, double *work, int *status,
                                                  double *rcond_out) {
  __shared__ double red[16];
  __shared__ double rv[1024];
  __shared__ int ri[1024];
  __shared__ int s_sing;
  __shared__ double s_anorm, s_est, s_done;
  const int tid = threadIdx.x, nt = blockDim.x;
  // ||A||_1 before factorisation (scipy computes lange('1') first)
  double cm = 0.0;
  for (int c = tid; c < n; c += nt) {
    double s = 0.0;
    for (int r = 0; r < n; ++r) s += fabs(A[(int64_t)r * n + c]);
    cm = fmax(cm, s);
  }
  rv[tid] = cm;
  __syncthreads();
  if (tid == 0) {
    double mx = 0.0;
    for (int i = 0; i < nt; ++i) mx = fmax(mx, rv[i]);
    s_anorm = mx;
    s_sing = 0;
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    // pivot: first index of max |A[i][j]|, i >= j
    double best = -1.0;
    int bi = j;
    for (int i = j + tid; i < n; i += nt) {
      const double v = fabs(A[(int64_t)i * n + j]);
      if (v > best) {
        best = v;
        bi = i;
      }
    }
    rv[tid] = best;
    ri[tid] = bi;
    __syncthreads();
    for (int s = nt / 2; s > 0; s >>= 1) {
      if (tid < s) {
        const double o = rv[tid + s];
        const int oi = ri[tid + s];
        if (o > rv[tid] || (o == rv[tid] && oi < ri[tid])) {
          rv[tid] = o;
          ri[tid] = oi;
        }
      }
      __syncthreads();
    }
    const int p = ri[0];
    if (tid == 0) piv[j] = p;
    if (p != j)
      for (int c = tid; c < n; c += nt) {
        const double t = A[(int64_t)j * n + c];
        A[(int64_t)j * n + c] = A[(int64_t)p * n + c];
        A[(int64_t)p * n + c] = t;
      }
    __syncthreads();
    const double d = A[(int64_t)j * n + j];
    if (d == 0.0) {
      if (tid == 0 && !s_sing) s_sing = j + 1;
      __syncthreads();
      continue;
    }
    const double inv = 1.0 / d;
    for (int i = j + 1 + tid; i < n; i += nt) A[(int64_t)i * n + j] *= inv;
    __syncthreads();
    const int t = n - j - 1;
    for (int64_t e = tid; e < (int64_t)t * t; e += nt) {
      const int i = j + 1 + (int)(e / t), c = j + 1 + (int)(e % t);
      A[(int64_t)i * n + c] -= A[(int64_t)i * n + j] * A[(int64_t)j * n + c];
    }
    __syncthreads();
  }
  if (s_sing) {
    if (tid == 0) {
      *status = s_sing;
      *rcond_out = 0.0;
    }
    return;
  }
  // Hager/Higham 1-norm estimate of ||A^-1||_1 (LAPACK gecon / lacn2 style)
  double *x = work, *xs = work + n;
  for (int i = tid; i < n; i += nt) x[i] = 1.0 / n;
  if (tid == 0) {
    s_est = 0.0;
    s_done = 0.0;
  }
  __syncthreads();
  int jlast = -1;
  for (int iter = 0; iter < 5; ++iter) {
    lu_vec_solve(A, n, piv, x, 0);
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
    lu_vec_solve(A, n, piv, xs, 1);
    // j = argmax |z|
    double best = -1.0;
    int bi = 0;
    for (int i = tid; i < n; i += nt)
      if (fabs(xs[i]) > best) {
        best = fabs(xs[i]);
        bi = i;
      }
    rv[tid] = best;
    ri[tid] = bi;
    __syncthreads();
    for (int s = nt / 2; s > 0; s >>= 1) {
      if (tid < s) {
        if (rv[tid + s] > rv[tid] || (rv[tid + s] == rv[tid] && ri[tid + s] < ri[tid])) {
          rv[tid] = rv[tid + s];
          ri[tid] = ri[tid + s];
        }
      }
      __syncthreads();
    }
    const int jn = ri[0];
    __syncthreads();
    if (jn == jlast) break;
    jlast = jn;
    for (int i = tid; i < n; i += nt) x[i] = (i == jn) ? 1.0 : 0.0;
    __syncthreads();
  }
  // alternating-sign test vector
  for (int i = tid; i < n; i += nt) x[i] = ((i & 1) ? -1.0 : 1.0) * (1.0 + (n > 1 ? (double)i / (n - 1) : 0.0));
  __syncthreads();
  lu_vec_solve(A, n, piv, x, 0);
  double s1 = 0.0;
  for (int i = tid; i < n; i += nt) s1 += fabs(x[i]);
  s1 = ttk::block_sum(s1, red);
  if (tid == 0) {
    const double temp = 2.0 * s1 / (3.0 * n);
    const double est = fmax(s_est, temp);
    *rcond_out = (s_anorm == 0.0 || est == 0.0) ? 0.0 : (1.0 / s_anorm) / est;
    *status = 0;
  }
}

// getrs on a matrix RHS: B (n x nrhs), each workgroup owns 64 columns
__global__ __launch_bounds__(256) void lu_solve_kernel(const double *__restrict__ LU, int n, const int *piv,
                                                       double *B, int nrhs, int ldb) {
  const int c0 = blockIdx.x * 64;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int ncol = min(64, nrhs - c0);
  if (ncol <= 0) return;
  for (int i = 0; i < n; ++i) {
    const int p = piv[i];
    if (p != i)
      for (int c = tid; c < ncol; c += nt) {
        const double t = B[(int64_t)i * ldb + c0 + c];
        B[(int64_t)i * ldb + c0 + c] = B[(int64_t)p * ldb + c0 + c];
        B[(int64_t)p * ldb + c0 + c] = t;
      }
    __syncthreads();
  }
  for (int i = 0; i < n; ++i) {
    const int rem = n - i - 1;
    for (int64_t e = tid; e < (int64_t)rem * ncol; e += nt) {
      const int r = i + 1 + (int)(e / ncol), c = (int)(e % ncol);
      B[(int64_t)r * ldb + c0 + c] -= LU[(int64_t)r * n + i] * B[(int64_t)i * ldb + c0 + c];
    }
    __syncthreads();
  }
  for (int i = n - 1; i >= 0; --i) {
    const double dinv = 1.0 / LU[(int64_t)i * n + i];
    for (int c = tid; c < ncol; c += nt) B[(int64_t)i * ldb + c0 + c] *= dinv;
    __syncthreads();
    for (int64_t e = tid; e < (int64_t)i * ncol; e += nt) {
      const int r = (int)(e / ncol), c = (int)(e % ncol);
      B[(int64_t)r * ldb + c0 + c] -= LU[(int64_t)r * n + i] * B[(int64_t)i * ldb + c0 + c];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------ SYEV (Jacobi)
__global__ __launch_bounds__(1024) void syev_kernel(double *__restrict__ Ain, int n, double *__restrict__ ev,
                                                    double *__restrict__ Wout, double *__restrict__ gwork,
                                                    int use_lds) {
  extern __shared__ double lds[];
  __shared__ int any_rot;
  double *A = use_lds ? lds : gwork;
  double *V = A + (int64_t)n * n;
  double *cs = V + (int64_t)n * n;  // c,s per pair (n/2+1 pairs) and pair indices
  double *d = cs + 2 * (n / 2 + 1);
  int *rank = reinterpret_cast<int *>(d + n);
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int64_t e = tid; e < (int64_t)n * n; e += nt) {
    A[e] = Ain[e];
    V[e] = ((e / n) == (e % n)) ? 1.0 : 0.0;
  }
  __syncthreads();
  const int P = (n % 2) ? n + 1 : n;
  __shared__ double red[16];
  double fro = 0.0;
  for (int64_t e = tid; e < (int64_t)n * n; e += nt) fro += A[e] * A[e];
  fro = sqrt(ttk::block_sum(fro, red));
  const double abs_floor = EPS * fro / (n > 1 ? n : 1);
  for (int sweep = 0; sweep < 40 && n > 1; ++sweep) {
    if (tid == 0) any_rot = 0;
    __syncthreads();
    for (int r = 0; r < P - 1; ++r) {
      // phase 0: rotation parameters from the current matrix
      for (int k = tid; k < P / 2; k += nt) {
        int p, q;
        rr_pair(P, r, k, p, q);
        double c = 1.0, s = 0.0;
        if (q < n) {
          const double apq = A[(int64_t)p * n + q];
          const double app = A[(int64_t)p * n + p], aqq = A[(int64_t)q * n + q];
          if (fabs(apq) > EPS * sqrt(fabs(app) * fabs(aqq)) && fabs(apq) > abs_floor && fabs(apq) > 1e-300) {
            const double th = (aqq - app) / (2.0 * apq);
            double t;
            if (fabs(th) > 1e150)
              t = 0.5 / th;
            else
              t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
            c = 1.0 / sqrt(t * t + 1.0);
            s = t * c;
            any_rot = 1;
          }
        }
        cs[2 * k] = c;
        cs[2 * k + 1] = s;
      }
      __syncthreads();
      // phase 1: rows  (J^T A)
      for (int64_t e = tid; e < (int64_t)(P / 2) * n; e += nt) {
        const int k = (int)(e / n), col = (int)(e % n);
        int p, q;
        rr_pair(P, r, k, p, q);
        if (q >= n) continue;
        const double c = cs[2 * k], s = cs[2 * k + 1];
        if (s == 0.0) continue;
        const double x = A[(int64_t)p * n + col], y = A[(int64_t)q * n + col];
        A[(int64_t)p * n + col] = c * x - s * y;
        A[(int64_t)q * n + col] = s * x + c * y;
      }
      __syncthreads();
      // phase 2: columns (A J) and eigenvectors (V J)
      for (int64_t e = tid; e < (int64_t)(P / 2) * n; e += nt) {
        const int k = (int)(e / n), row = (int)(e % n);
        int p, q;
        rr_pair(P, r, k, p, q);
        if (q >= n) continue;
        const double c = cs[2 * k], s = cs[2 * k + 1];
        if (s == 0.0) continue;
        double x = A[(int64_t)row * n + p], y = A[(int64_t)row * n + q];
        A[(int64_t)row * n + p] = c * x - s * y;
        A[(int64_t)row * n + q] = s * x + c * y;
        x = V[(int64_t)row * n + p];
        y = V[(int64_t)row * n + q];
        V[(int64_t)row * n + p] = c * x - s * y;
        V[(int64_t)row * n + q] = s * x + c * y;
      }
      __syncthreads();
    }
    if (!any_rot) break;
    __syncthreads();
  }
  for (int i = tid; i < n; i += nt) d[i] = A[(int64_t)i * n + i];
  __syncthreads();
  for (int j = tid; j < n; j += nt) {
    int rk = 0;
    const double dj = d[j];
    for (int i = 0; i < n; ++i) rk += (d[i] < dj) || (d[i] == dj && i < j);
    rank[j] = rk;
  }
  __syncthreads();
  for (int j = tid; j < n; j += nt) ev[rank[j]] = d[j];
  for (int64_t e = tid; e < (int64_t)n * n; e += nt) {
    const int i = (int)(e / n), j = (int)(e % n);
    Wout[(int64_t)i * n + rank[j]] = V[e];
  }
}

template <typename K>
void allow_big_lds(K kernel, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

int *g_status = nullptr;
double *g_rcond = nullptr;

int ensure_status() {
  if (!g_status) {
    if (hipMalloc(reinterpret_cast<void **>(&g_status), 16 * sizeof(int)) != hipSuccess) return TTK_ERR_HIP;
    if (hipMalloc(reinterpret_cast<void **>(&g_rcond), 16 * sizeof(double)) != hipSuccess) return TTK_ERR_HIP;
  }
  return TTK_OK;
}

}  // namespace

extern "C" {

int64_t ttk_svd_work(int m, int n) {
  const int64_t p = m < n ? m : n, q = m < n ? n : m;
  return q * p + p * p + 2 * p + 16;
}

int ttk_svd(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt, double *work) {
  if (m <= 0 || n <= 0) {
    ttk::set_error("ttk_svd: empty matrix %dx%d", m, n);
    return TTK_ERR_ARG;
  }
  const int64_t need = ttk_svd_work(m, n);
  const int use_lds = need <= LDS_DOUBLES;
  const size_t shm = use_lds ? need * sizeof(double) : 0;
  allow_big_lds(svd_kernel, shm);
  hipLaunchKernelGGL(svd_kernel, dim3(1), dim3(1024), shm, TTK_STREAM(stream), A, m, n, U, S, Vt, work, use_lds);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int64_t ttk_qr_work(int m, int n) {
  const int64_t k = m < n ? m : n;
  return (int64_t)m * n + k + (int64_t)m * k + 16;
}

int ttk_qr(void *stream, const double *A, int m, int n, double *Q, double *R, double *work) {
  if (m <= 0 || n <= 0) {
    ttk::set_error("ttk_qr: empty matrix %dx%d", m, n);
    return TTK_ERR_ARG;
  }
  const int64_t need = ttk_qr_work(m, n);
  const int use_lds = need <= LDS_DOUBLES;
  const size_t shm = use_lds ? need * sizeof(double) : 0;
  allow_big_lds(qr_kernel, shm);
  hipLaunchKernelGGL(qr_kernel, dim3(1), dim3(1024), shm, TTK_STREAM(stream), A, m, n, Q, R, work, use_lds);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_cholesky_sync(void *stream, double *A, int n) {
  if (ensure_status()) {
    ttk::set_error("ttk_cholesky_sync: status alloc failed");
    return TTK_ERR_HIP;
  }
  hipLaunchKernelGGL(chol_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), A, n, g_status);
  TTK_LAUNCH_CHECK();
  int st = 0;
  TTK_HIP(hipMemcpyAsync(&st, g_status, sizeof(int), hipMemcpyDeviceToHost, TTK_STREAM(stream)));
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  if (st) {
    ttk::set_error("%d-th leading minor of the array is not positive definite", st);
    return TTK_ERR_NOT_PD;
  }
  return TTK_OK;
}

int ttk_trsm_lower(void *stream, const double *L, int n, double *B, int nrhs, int ldb, int trans) {
  if (n <= 0 || nrhs <= 0) return TTK_OK;
  hipLaunchKernelGGL(trsm_kernel, dim3((nrhs + 63) / 64), dim3(256), 0, TTK_STREAM(stream), L, n, B, nrhs, ldb, trans);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_lu_sync(void *stream, double *A, int n, int *piv, double *work, double *rcond_out) {
  if (ensure_status()) {
    ttk::set_error("ttk_lu_sync: status alloc failed");
    return TTK_ERR_HIP;
  }
  hipLaunchKernelGGL(lu_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), A, n, piv, work, g_status, g_rcond);
  TTK_LAUNCH_CHECK();
  int st = 0;
  TTK_HIP(hipMemcpyAsync(&st, g_status, sizeof(int), hipMemcpyDeviceToHost, TTK_STREAM(stream)));
  TTK_HIP(hipMemcpyAsync(rcond_out, g_rcond, sizeof(double), hipMemcpyDeviceToHost, TTK_STREAM(stream)));
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  if (st) {
    ttk::set_error("Matrix is singular (zero pivot at %d).", st);
    return TTK_ERR_SINGULAR;
  }
  return TTK_OK;
}

int ttk_lu_solve(void *stream, const double *LU, int n, const int *piv, double *B, int nrhs, int ldb) {
  if (n <= 0 || nrhs <= 0) return TTK_OK;
  hipLaunchKernelGGL(lu_solve_kernel, dim3((nrhs + 63) / 64), dim3(256), 0, TTK_STREAM(stream), LU, n, piv, B, nrhs, ldb);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int64_t ttk_syev_work(int n) { return 2 * (int64_t)n * n + 2 * (n / 2 + 1) + 2 * (int64_t)n + 16; }

int ttk_syev(void *stream, double *A, int n, double *ev, double *W, double *work) {
  if (n <= 0) {
    ttk::set_error("ttk_syev: empty matrix");
    return TTK_ERR_ARG;
  }
  const int64_t need = ttk_syev_work(n);
  const int use_lds = need <= LDS_DOUBLES;
  const size_t shm = use_lds ? need * sizeof(double) : 0;
  allow_big_lds(syev_kernel, shm);
  hipLaunchKernelGGL(syev_kernel, dim3(1), dim3(1024), shm, TTK_STREAM(stream), A, n, ev, W, work, use_lds);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

}  // extern "C"
