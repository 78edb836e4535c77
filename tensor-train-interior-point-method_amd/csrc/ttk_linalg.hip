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
#include <stdlib.h>

#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>

#include "ttk_common.h"
#include "ttk_internal.h"

namespace {

constexpr double EPS = 2.220446049250313e-16;
// diagnostic counters: [0] svd calls, [1] svd sweeps, [2] eig calls, [3] multisection rounds,
// [4..7] one-workgroup SVD phase ticks (QRCP, Jacobi, vectors, output; 100 MHz)
__device__ unsigned long long g_dbg[8];

constexpr int LDS_DOUBLES = 20000;  // 160000 B of dynamic LDS (gfx950: 160 KiB per workgroup)

// round-robin (circle method) pair k of round r over P (even) items; 0 <= r < P-1, 0 <= k < P/2,
// so both residues need one conditional subtraction (a runtime-divisor `%` costs ~280 cycles)
__device__ __forceinline__ void rr_pair(int P, int r, int k, int &p, int &q) {
  const int P1 = P - 1;
  if (k == 0) {
    p = r;
    q = P1;
  } else {
    p = r + k;
    if (p >= P1) p -= P1;
    q = r - k + P1;
    if (q >= P1) q -= P1;
  }
  if (p > q) {
    int t = p;
    p = q;
    q = t;
  }
}

// 1/x and 1/sqrt(x) from the hardware estimates plus Newton steps (~1 ulp).  Rotation parameters
// only need c^2 + s^2 = 1 to a few ulps; the IEEE div/sqrt expansions cost ~280 cycles each.
__device__ __forceinline__ double fast_rcp(double x) {
#ifdef TTK_EXACT_DIV
  return 1.0 / x;
#endif
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  r = fma(fma(-x, r, 1.0), r, r);
  return r;
}

__device__ __forceinline__ double fast_rsqrt(double x) {
#ifdef TTK_EXACT_DIV
  return 1.0 / sqrt(x);
#endif
  double r = __builtin_amdgcn_rsq(x);
  double h = 0.5 * x * r;
  double e = fma(-h, r, 0.5);
  r = fma(r, e, r);
  h = 0.5 * x * r;
  e = fma(-h, r, 0.5);
  return fma(r, e, r);
}

// Hestenes rotation zeroing the pair's inner product ga (column norms^2 al, be):
// t = sign(d) 2 ga / (|d| + sqrt(d^2 + 4 ga^2)), d = be - al; c = 1/sqrt(1 + t^2), s = c t.
// (Same t as Rutishauser's zeta form, without the zeta division and its overflow branch.)
__device__ __forceinline__ void jacobi_rotation(double al, double be, double ga, double &c, double &s) {
  const double d = be - al, g2 = 2.0 * ga;
  const double hh = fma(d, d, g2 * g2);
  const double h = hh * fast_rsqrt(hh);  // sqrt(d^2 + 4 ga^2) > 0 since ga != 0
  double t = g2 * fast_rcp(fabs(d) + h);
  if (d < 0.0) t = -t;
  c = fast_rsqrt(fma(t, t, 1.0));
  s = c * t;
}

// ------------------------------------------------------------------------------ SVD
// W: q x p column-major (column j at W + j*q), V: p x p column-major.
// Shared epilogue of both SVD paths (one workgroup): singular values = column norms of the
// converged W, descending order, unit left vectors (exact-zero columns completed), outputs.
__device__ void svd_epilogue(double *W, double *V, double *sig, int *rank, int m, int n, bool tall,
                             double *__restrict__ U, double *__restrict__ S, double *__restrict__ Vt) {
  __shared__ double red[16];
  const int p = tall ? n : m, q = tall ? m : n;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  // singular values = column norms
  for (int j = wid; j < p; j += nw) {
    const double *wj = W + (int64_t)j * q;
    double s2 = 0.0;
    #pragma unroll 8
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
      #pragma unroll 8
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

// Multi-workgroup one-sided Jacobi for large unfoldings (the 1e-12 rank reductions at the end of
// a solve produce ~1000 x 1000 swap/rounding unfoldings), run on X = R^T after a blocked QR
// (svd_big below).  One wave per column pair, one launch per round-robin round (all P/2 pairs in
// flight across the chip); X and V stay L2/MALL resident.  The host drives sweeps and reads one
// convergence flag per sweep.
__global__ __launch_bounds__(256) void svd_big_round_kernel(double *__restrict__ W, double *__restrict__ V, int p,
                                                            int q, int r, double tol, int *__restrict__ flag) {
  const int P = (p % 2) ? p + 1 : p;
  const int k = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= P / 2) return;  // whole wave exits together
  int a, b;
  rr_pair(P, r, k, a, b);
  if (b >= p) return;
  double *wa = W + (int64_t)a * q, *wb = W + (int64_t)b * q;
  double al = 0.0, be = 0.0, ga = 0.0;
  #pragma unroll 8
  for (int i = lane; i < q; i += 64) {
    const double x = wa[i], y = wb[i];
    al += x * x;
    be += y * y;
    ga += x * y;
  }
  al = ttk::wave_sum(al);
  be = ttk::wave_sum(be);
  ga = ttk::wave_sum(ga);
  if (al < 1e-300 || be < 1e-300) return;
  if (ga * ga <= tol * tol * al * be) return;
  double c, s;
  jacobi_rotation(al, be, ga, c, s);
  #pragma unroll 8
  for (int i = lane; i < q; i += 64) {
    const double x = wa[i], y = wb[i];
    wa[i] = c * x - s * y;
    wb[i] = s * x + c * y;
  }
  double *va = V + (int64_t)a * p, *vb = V + (int64_t)b * p;
  #pragma unroll 8
  for (int i = lane; i < p; i += 64) {
    const double x = va[i], y = vb[i];
    va[i] = c * x - s * y;
    vb[i] = s * x + c * y;
  }
  if (lane == 0) *flag = 1;
}

// One launch per Jacobi SWEEP instead of per round (TTK_KNOB_SVD_SWEEP_ONE): the P/2 pair waves of
// svd_big_round_kernel stay resident for all P-1 rounds of the sweep, and a wave starts its pair of
// round r as soon as its two columns have finished round r-1 -- per-column round counters `colr`
// (in-launch hand-offs, ttk_common.h: sc1 stores, drain, agent-scope release; the consumer polls, then
// acquires and loads with sc1), no grid-wide barrier.  Each column belongs to exactly one pair per
// round, so a column's rounds are totally ordered through its counter, and every rotation is
// svd_big_round_kernel's: the same expressions on the same values in the same round order
// (bit-identical, tools/dump_kernels.py).  The wave's pair index is its workgroup's start ticket x 4
// + its wave index.  A wave waits only for waves of the previous round, which wait only for earlier
// rounds; round 0 never waits, so with every workgroup resident the launch drains -- the grid is
// P/8 <= 256 workgroups of 256 threads, far below the chip's resident capacity, and a poll past
// DEP_SPIN_MAX gives up and is counted (dep[1], ttk_dep_timeouts) instead of hanging.
// colr[c] = base + (rounds of this sweep column c has finished); the host zeroes colr per SVD and
// passes base = sweep * (P - 1).
__device__ __forceinline__ void colr_wait(const unsigned *colr, int a, int b, unsigned target, unsigned *dep) {
  if ((threadIdx.x & 63) == 0) {
    const __attribute__((address_space(1))) unsigned *ca = (const __attribute__((address_space(1))) unsigned *)(colr + a);
    const __attribute__((address_space(1))) unsigned *cb = (const __attribute__((address_space(1))) unsigned *)(colr + b);
    long n = 0;
    while ((int)(__hip_atomic_load(ca, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0 ||
           (int)(__hip_atomic_load(cb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++n > ttk::DEP_SPIN_MAX) {
        __hip_atomic_fetch_add(dep + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
#ifndef TTK_HANDOFF_RELAXED
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // no column load moves above the poll
}

__global__ __launch_bounds__(256) void svd_big_sweep_kernel(double *__restrict__ W, double *__restrict__ V, int p,
                                                            int q, double tol, int *__restrict__ flag, unsigned *colr,
                                                            unsigned base, unsigned *dep, unsigned tick_base) {
  const int P = (p % 2) ? p + 1 : p;
  const int k = ttk::ticket(dep, tick_base) * 4 + (int)(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= P / 2) return;  // whole wave exits together (no pair: nobody waits for it)
  bool rot = false;
  for (int r = 0; r < P - 1; ++r) {
    int a, b;
    rr_pair(P, r, k, a, b);
    colr_wait(colr, a, b, base + (unsigned)r, dep);
    if (b < p) {
      double *wa = W + (int64_t)a * q, *wb = W + (int64_t)b * q;
      double al = 0.0, be = 0.0, ga = 0.0;
#pragma unroll 8
      for (int i = lane; i < q; i += 64) {
        const double x = ttk::ld_sc1(wa + i), y = ttk::ld_sc1(wb + i);
        al += x * x;
        be += y * y;
        ga += x * y;
      }
      al = ttk::wave_sum(al);
      be = ttk::wave_sum(be);
      ga = ttk::wave_sum(ga);
      if (!(al < 1e-300 || be < 1e-300) && !(ga * ga <= tol * tol * al * be)) {
        double c, s;
        jacobi_rotation(al, be, ga, c, s);
#pragma unroll 8
        for (int i = lane; i < q; i += 64) {
          const double x = ttk::ld_sc1(wa + i), y = ttk::ld_sc1(wb + i);
          ttk::st_sc1(wa + i, c * x - s * y);
          ttk::st_sc1(wb + i, s * x + c * y);
        }
        double *va = V + (int64_t)a * p, *vb = V + (int64_t)b * p;
#pragma unroll 8
        for (int i = lane; i < p; i += 64) {
          const double x = ttk::ld_sc1(va + i), y = ttk::ld_sc1(vb + i);
          ttk::st_sc1(va + i, c * x - s * y);
          ttk::st_sc1(vb + i, s * x + c * y);
        }
        rot = true;
      }
    }
    // publish both columns' round r: drain the sc1 stores, release, then the counters
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifndef TTK_HANDOFF_RELAXED
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    if (lane == 0) {
      __hip_atomic_store(colr + a, base + (unsigned)r + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(colr + b, base + (unsigned)r + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (rot && lane == 0) *flag = 1;
}

__global__ __launch_bounds__(1024) void svd_big_finish_kernel(double *W, double *V, double *sig, int *rank, int m,
                                                              int n, double *__restrict__ U, double *__restrict__ S,
                                                              double *__restrict__ Vt) {
  svd_epilogue(W, V, sig, rank, m, n, m >= n, U, S, Vt);
}

// ------------------------------------------- one-workgroup SVD with QRCP preconditioning
// For min(m,n) <= WG_P: W = A (tall) or A^T (wide), q x p column-major.  W P = Q R by column-
// pivoted Householder QR inside the workgroup (pivot/reflector by wave 0, one wave per trailing
// column with the dlaqp2 norm downdate), then one-sided Jacobi on X = R1^T (p x kk) with X and V
// resident in LDS, then the left vectors Q [V_X; 0] (one wave per column through all
// reflectors, no block barriers) and the right vectors P U_X.  QRCP grades the rows of R, which
// cuts the Jacobi sweeps ~4x on the path's unfoldings and shrinks the column length from q to p.
constexpr int WG_P = 96;


// One round-robin round of one-sided Jacobi with G lanes per column pair; each lane keeps its
// <= VPL elements of both columns in registers for the whole round (one LDS load batch, one
// store batch), so a round costs ~two LDS latencies plus the rotation instead of one LDS round
// trip per element.
constexpr int VPL = 8;

template <int G>
__device__ __forceinline__ void jacobi_round(double *X, int ldx, double *V, int ldv, int p, int L, int P, int r,
                                             double tol2, int *any_rot) {
  const int tid = threadIdx.x, gl = tid & (G - 1), gid = tid / G, ng = blockDim.x / G;
  for (int k = gid; k < P / 2; k += ng) {
    int a, b;
    rr_pair(P, r, k, a, b);
    if (b >= p) continue;
    double *wa = X + a * ldx, *wb = X + b * ldx;
    double *va = V + a * ldv, *vb = V + b * ldv;
    double xa[VPL], xb[VPL], ya[VPL], yb[VPL];
    // both columns of X and of V in one batch of LDS loads (the V columns used to be loaded after
    // the X stores, one more LDS round trip per round; the pair owns all four columns this round)
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int i = gl + v * G;
      xa[v] = i < L ? wa[i] : 0.0;
      xb[v] = i < L ? wb[i] : 0.0;
      ya[v] = i < p ? va[i] : 0.0;
      yb[v] = i < p ? vb[i] : 0.0;
    }
    double al = 0.0, be = 0.0, ga = 0.0;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      al = fma(xa[v], xa[v], al);
      be = fma(xb[v], xb[v], be);
      ga = fma(xa[v], xb[v], ga);
    }
    if (G > 1) {
      al = ttk::group_sum_rt(al, G);
      be = ttk::group_sum_rt(be, G);
      ga = ttk::group_sum_rt(ga, G);
    }
    if (al < 1e-300 || be < 1e-300) continue;
    if (ga * ga <= tol2 * al * be) continue;  // |ga| <= tol sqrt(al be)
    double cs, sn;
    jacobi_rotation(al, be, ga, cs, sn);
    // the rotations with the contractions the compiler chose for the previous form of this loop
    // (wa, wb, va: the product of the second term first; vb: of the first), spelled out so that
    // moving the loads cannot change them
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int i = gl + v * G;
      if (i < L) {
        wa[i] = fma(cs, xa[v], -(sn * xb[v]));
        wb[i] = fma(cs, xb[v], sn * xa[v]);
      }
    }
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int i = gl + v * G;
      if (i < p) {
        va[i] = fma(cs, ya[v], -(sn * yb[v]));
        vb[i] = fma(sn, ya[v], cs * yb[v]);
      }
    }
    if (gl == 0) *any_rot = 1;
  }
}

// WM: where the QRCP working copy W and the left-vector buffer M live -- 2 both in LDS, 1 W in LDS and
// M in global memory, 0 both global -- known at compile time so that their accesses are LDS
// instructions, not flat ones (a flat access waits on both the LDS and the vector-memory counters)
template <int G, int WM>
__global__ __launch_bounds__(1024) void svd_wg_kernel(const double *__restrict__ A, int m, int n,
                                                      double *__restrict__ U, double *__restrict__ S,
                                                      double *__restrict__ Vt, double *__restrict__ gwork,
                                                      int w_in_lds, int use_qr, int timing,
                                                      double *__restrict__ host_s) {
  extern __shared__ double lds[];
  constexpr bool WL = WM >= 1, ML = WM == 2;  // W in LDS; M in LDS too
  constexpr int SU = ML ? 8 : 4;  // loads ahead in the dot chains (W or M in global memory: fewer registers left)
  __shared__ int s_piv, any_rot;
  __shared__ double red[16];
  const bool tall = m >= n;
  const int p = tall ? n : m, q = tall ? m : n;
  const int L = use_qr ? p : q;  // Jacobi column length
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  unsigned long long t_ph = timing ? wall_clock64() : 0;
  const unsigned long long t_w0 = t_ph, t_c0 = timing ? clock64() : 0;  // shader clock vs 100 MHz wall
#define TTK_PHASE(K)                                    \
  if (timing && tid == 0) {                             \
    const unsigned long long t1 = wall_clock64();       \
    atomicAdd(&g_dbg[K], t1 - t_ph);                    \
    t_ph = t1;                                          \
  }
  // LDS: X (ldx*p) | V (ldv*p) | tau, vn1, vn2, sig (4p) | perm, rank (2p ints) | [W (WM >= 1), M (WM == 2)]
  // odd leading dimensions: columns start on different LDS banks (even ones put every lane group
  // of a wave on the same banks)
  const int ldx = L | 1, ldv = p | 1;
  // g2 lanes per column for the column-parallel QR phases: as many as fill the block, <= 64
  int g2 = 64;
  while (g2 > 1 && g2 * (p > 1 ? p - 1 : 1) > nt) g2 >>= 1;
  const int gl2 = tid & (g2 - 1), gid2 = tid / g2, ng2 = nt / g2;
  double *X = lds, *V = X + ldx * p, *tau = V + ldv * p, *vn1 = tau + p, *vn2 = vn1 + p, *sig = vn2 + p;
  int *perm = reinterpret_cast<int *>(sig + p), *rank = perm + p;
  // W right after the 2p ints of perm / rank: 8-byte aligned for any p (an extra int for odd p, as
  // before round 5, put every double of W and M on a 4-byte boundary -- each ds_read/write_b64 then
  // took the misaligned path: QRCP's trailing update and the left-vector pass ran 3-6x slower per
  // element for odd p, SQ_LDS_IDX_ACTIVE 1.8M vs 0.34M cycles at 64 x 63 vs 144 x 48)
  double *W = use_qr ? (WL ? reinterpret_cast<double *>(rank + p) : gwork) : X;
  // W / M column stride: odd, so the g2-lane groups of one wave (consecutive columns) start on
  // different LDS banks (an even q put every group of a wave on the same banks)
  const int lq = q | 1;
  const int ldw = use_qr ? lq : ldx;
  // M after W where both are in the same memory; WM = 1 (W fits LDS, W and M together do not): M is
  // the global working buffer -- the QRCP then runs on LDS, only the left-vector pass on global memory
  double *M = (ML || !WL) ? W + (int64_t)lq * p : gwork;
  for (int e = tid; e < q * p; e += nt) {
    const int j = e / q, i = e - j * q;
    W[(int64_t)j * ldw + i] = tall ? A[(int64_t)i * n + j] : A[(int64_t)j * n + i];
  }
  __syncthreads();
  if (use_qr) {
    for (int j = wid; j < p; j += nw) {
      const double *w = W + (int64_t)j * lq;
      double acc = ttk::chain_ahead<SU>(
          ttk::steps_below(lane, q, 64), [&](int k) { return w[lane + 64 * k]; },
          [&](int k) { return w[lane + 64 * k]; }, 0.0);
      acc = sqrt(ttk::wave_sum(acc));
      if (lane == 0) {
        vn1[j] = acc;
        vn2[j] = acc;
        perm[j] = j;
      }
    }
    __syncthreads();
    // ---- QRCP (all p steps: zero columns get tau = 0, so every direction keeps a unit vector).
    // Two block barriers per column: every wave picks the pivot itself (the same first max of the
    // same downdated norms), wave 0 swaps the pivot column into place and builds the reflector,
    // barrier, trailing update + norm downdate, barrier.  The vn1 / vn2 / perm swap is folded into
    // the trailing phase (slot piv takes slot c's values; slot c is never read again), so no wave
    // writes the norms while another still reads them for its pivot search.
    for (int c = 0; c < p; ++c) {
      int piv;
      {  // first max of the downdated norms (idamax) over <= 96 columns, every wave
        double bm = -1.0;
        int bi = p;
        for (int j = c + lane; j < p; j += 64) {
          const double v = vn1[j];
          if (v > bm) {
            bm = v;
            bi = j;
          }
        }
        ttk::wave_argmax(bm, bi);  // first max of the downdated norms, DPP (same winner as a butterfly)
        piv = bi < p ? bi : c;
      }
      double *x = W + (int64_t)c * lq;
      if (wid == 0) {  // pivot swap + reflector (dlarfg) by wave 0 (LDS ops of one wave stay in order)
        if (piv != c) {
          double *b = W + (int64_t)piv * lq;
          for (int i = lane; i < q; i += 64) {
            const double t = x[i];
            x[i] = b[i];
            b[i] = t;
          }
        }
        const double part = ttk::chain_ahead<SU>(
            ttk::steps_below(c + 1 + lane, q, 64), [&](int k) { return x[c + 1 + lane + 64 * k]; },
            [&](int k) { return x[c + 1 + lane + 64 * k]; }, 0.0);
        const double sigma = ttk::wave_sum(part);
        const double alpha = x[c];
        double t = 0.0, beta = alpha;
        if (sigma > 0.0) {
          beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
          t = (beta - alpha) / beta;
          const double sc = 1.0 / (alpha - beta);
          #pragma unroll 8
          for (int i = c + 1 + lane; i < q; i += 64) x[i] *= sc;
        }
        if (lane == 0) {
          x[c] = beta;
          tau[c] = t;
          if (piv != c) {
            const int pi = perm[c];
            perm[c] = perm[piv];
            perm[piv] = pi;
          }
        }
      }
      __syncthreads();
      const double t = tau[c];
      // trailing update + dlaqp2 norm downdate: g2 lanes per column, all columns in flight; column
      // piv carries slot c's norms after the swap
      for (int j = c + 1 + gid2; j < p; j += ng2) {
        double *y = W + (int64_t)j * lq;
        double yc = y[c];
        if (t != 0.0) {
          const double acc = ttk::chain_ahead<SU>(
              ttk::steps_below(c + 1 + gl2, q, g2), [&](int k) { return x[c + 1 + gl2 + g2 * k]; },
              [&](int k) { return y[c + 1 + gl2 + g2 * k]; }, 0.0);
          const double w = t * (ttk::group_sum_rt(acc, g2) + yc);
          ttk::axpy_sub_strided(y, x, w, c + 1 + gl2, q, g2);
          yc -= w;
          if (gl2 == 0) y[c] = yc;
        }
        const int js = j == piv ? c : j;
        const double a = vn1[js], a2 = vn2[js];
        if (a != 0.0) {
          double temp = fabs(yc) / a;
          temp = fmax(1.0 - temp * temp, 0.0);
          const double r = a / a2;
          if (temp * r * r <= 1.4901161193847656e-08) {
            __threadfence_block();  // the group reads back the updated column
            double acc = ttk::chain_ahead<SU>(
                ttk::steps_below(c + 1 + gl2, q, g2), [&](int k) { return y[c + 1 + gl2 + g2 * k]; },
                [&](int k) { return y[c + 1 + gl2 + g2 * k]; }, 0.0);
            acc = sqrt(ttk::group_sum_rt(acc, g2));
            if (gl2 == 0) {
              vn1[j] = acc;
              vn2[j] = acc;
            }
          } else if (gl2 == 0) {
            vn1[j] = a * sqrt(temp);
            vn2[j] = a2;
          }
        } else if (gl2 == 0 && j == piv) {
          vn1[j] = a;
          vn2[j] = a2;
        }
      }
      __syncthreads();
    }
    // X = R^T (column length p)
    for (int e = tid; e < p * p; e += nt) {
      const int i = e / p, j = e - i * p;
      X[i * ldx + j] = (j >= i) ? W[(int64_t)j * lq + i] : 0.0;
    }
  }
  for (int e = tid; e < p * p; e += nt) {
    const int j = e / p, i = e - j * p;
    V[j * ldv + i] = (i == j) ? 1.0 : 0.0;
  }
  __syncthreads();
  TTK_PHASE(4)
  // ---- one-sided Jacobi on the p columns of X (length L)
  const int P = (p % 2) ? p + 1 : p;
  const double tol = EPS * (L > 16 ? (double)L : 16.0), tol2 = tol * tol;
  for (int sweep = 0; sweep < 60 && p > 1; ++sweep) {
    if (tid == 0) any_rot = 0;
    __syncthreads();
    for (int r = 0; r < P - 1; ++r) {
      jacobi_round<G>(X, ldx, V, ldv, p, L, P, r, tol2, &any_rot);
      __syncthreads();
    }
    if (timing && tid == 0) atomicAdd(&g_dbg[1], 1ull);
    if (!any_rot) break;
    __syncthreads();
  }
  TTK_PHASE(5)
  // ---- singular values, order, unit columns
  for (int j = wid; j < p; j += nw) {
    const double *xj = X + j * ldx;
    double s2 = 0.0;
    for (int i = lane; i < L; i += 64) s2 += xj[i] * xj[i];
    s2 = ttk::wave_sum(s2);
    if (lane == 0) sig[j] = sqrt(s2);
  }
  __syncthreads();
  for (int j = tid; j < p; j += nt) {
    int rk = 0;
    const double sj = sig[j];
    for (int i = 0; i < p; ++i) rk += (sig[i] > sj) || (sig[i] == sj && i < j);
    rank[j] = rk;
  }
  __syncthreads();
  for (int j = wid; j < p; j += nw) {
    double *xj = X + j * ldx;
    const double sj = sig[j];
    const double inv = sj > 0.0 ? 1.0 / sj : 0.0;
    for (int i = lane; i < L; i += 64) xj[i] *= inv;
  }
  __syncthreads();
  // exact-zero columns: complete to an orthonormal set (rare; MGS against e_i candidates)
  for (int j = 0; j < p; ++j) {
    if (sig[j] > 0.0) continue;
    double *xj = X + j * ldx;
    for (int cand = 0; cand < L; ++cand) {
      for (int i = tid; i < L; i += nt) xj[i] = (i == cand) ? 1.0 : 0.0;
      __syncthreads();
      for (int o = 0; o < p; ++o) {
        if (o == j || (sig[o] == 0.0 && o > j)) continue;
        const double *xo = X + o * ldx;
        double d = 0.0;
        for (int i = tid; i < L; i += nt) d += xo[i] * xj[i];
        d = ttk::block_sum(d, red);
        for (int i = tid; i < L; i += nt) xj[i] -= d * xo[i];
        __syncthreads();
      }
      double nn = 0.0;
      for (int i = tid; i < L; i += nt) nn += xj[i] * xj[i];
      nn = ttk::block_sum(nn, red);
      if (nn > 0.25) {
        const double inv = 1.0 / sqrt(nn);
        for (int i = tid; i < L; i += nt) xj[i] *= inv;
        __syncthreads();
        break;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  TTK_PHASE(6)
  for (int j = tid; j < p; j += nt) S[rank[j]] = sig[j];
  if (host_s)  // the caller's host-coherent copy of S (a rank decision waits on it; no read kernel)
    for (int j = tid; j < p; j += nt) host_s[rank[j]] = sig[j];
  if (use_qr) {
    // left factor of W: M(:, rank[j]) = Q [V(:, j); 0]; g2 lanes per column, each column runs
    // through all reflectors independently (no block barriers)
    for (int j = gid2; j < p; j += ng2) {
      double *mc = M + (int64_t)rank[j] * lq;
      const double *vj = V + j * ldv;
      #pragma unroll 8
      for (int i = gl2; i < q; i += g2) mc[i] = i < p ? vj[i] : 0.0;
      __threadfence_block();
      for (int c = p - 1; c >= 0; --c) {
        const double t = tau[c];
        if (t == 0.0) continue;
        const double *v = W + (int64_t)c * lq;
        const double acc = ttk::chain_ahead<SU>(
            ttk::steps_below(c + 1 + gl2, q, g2), [&](int k) { return v[c + 1 + gl2 + g2 * k]; },
            [&](int k) { return mc[c + 1 + gl2 + g2 * k]; }, 0.0);
        const double w = t * (ttk::group_sum_rt(acc, g2) + mc[c]);
        ttk::axpy_sub_strided(mc, v, w, c + 1 + gl2, q, g2);
        __threadfence_block();
        if (gl2 == 0) mc[c] -= w;
        __threadfence_block();
      }
    }
  }
  __syncthreads();
  TTK_PHASE(7)
  // ---- outputs
  if (use_qr) {  // left = M (q x p), right(perm[i], rank[j]) = X(i, j)
    for (int e = tid; e < q * p; e += nt) {
      const int i = e / p, r = e - i * p;
      const double v = M[(int64_t)r * lq + i];
      if (tall)
        U[(int64_t)i * p + r] = v;
      else
        Vt[(int64_t)r * q + i] = v;
    }
    for (int e = tid; e < p * p; e += nt) {
      const int j = e / p, i = e - j * p;  // X(i, j): pivoted row i, column j
      const int r = rank[j], oi = perm[i];
      const double v = X[j * ldx + i];
      if (tall)
        Vt[(int64_t)r * p + oi] = v;
      else
        U[(int64_t)oi * p + r] = v;
    }
  } else {  // left(i, rank[j]) = X(i, j) (length q), right(i, rank[j]) = V(i, j)
    for (int e = tid; e < q * p; e += nt) {
      const int j = e / q, i = e - j * q;
      const double v = X[j * ldx + i];
      if (tall)
        U[(int64_t)i * p + rank[j]] = v;
      else
        Vt[(int64_t)rank[j] * q + i] = v;
    }
    for (int e = tid; e < p * p; e += nt) {
      const int j = e / p, i = e - j * p;
      const double v = V[j * ldv + i];
      if (tall)
        Vt[(int64_t)rank[j] * p + i] = v;
      else
        U[(int64_t)i * p + rank[j]] = v;
    }
  }
  if (timing) {  // (the output copies are not a phase of their own: a few us)
    __syncthreads();
    if (tid == 0) {
      atomicAdd(&g_dbg[0], 1ull);
      atomicAdd(&g_dbg[2], clock64() - t_c0);
      atomicAdd(&g_dbg[3], wall_clock64() - t_w0);
    }
  }
#undef TTK_PHASE
}

// ------------------------------------------------------------------------------ QR
// W: m x n column-major working copy; tau: k.
// UL: the working copy in LDS (use_lds), at compile time: LDS instructions instead of flat ones
template <bool UL>
// colmajor: A arrives column-major (A^T row-major) and Q leaves as Q^T row-major -- the layouts the
// TT rounding's right-to-left sweep holds, so it needs no transposing copies around the call; only
// the loads and stores differ, the arithmetic is the same
__global__ __launch_bounds__(1024) void qr_kernel(const double *__restrict__ A, int m, int n,
                                                  double *__restrict__ Q, double *__restrict__ R,
                                                  double *__restrict__ gwork, int use_lds, int colmajor) {
  extern __shared__ double lds[];
  constexpr int CU = UL ? 8 : 4;  // loads ahead in the dot chains
  __shared__ double red[16];
  __shared__ double s_beta, s_tau, s_scale;
  const int k = m < n ? m : n;
  double *W = UL ? lds : gwork;
  double *tau = W + (int64_t)m * n;
  double *Qc = tau + k;  // m x k column-major accumulation
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  for (int64_t e = tid; e < (int64_t)m * n; e += nt) {
    const int j = (int)(e / m), i = (int)(e % m);
    W[e] = colmajor ? A[e] : A[(int64_t)i * n + j];
  }
  __syncthreads();
  if (m <= 65) {
    // every lane holds at most one element of column j below the diagonal, so each wave can form the
    // reflector itself: the norm is wave 0's wave sum in the block-wide path (the other waves add
    // zeros), the scaled vector stays in registers, and each wave updates the columns it owns (c % nw
    // == wid) -- one block barrier per column instead of four.  The same operations on every element
    // in the same order as the block-wide loop below: bit-identical
    for (int j = 0; j < k; ++j) {
      double *wj = W + (int64_t)j * m;
      const int i = j + 1 + lane;
      const double x = i < m ? wj[i] : 0.0;
      const double s2 = 0.0 + ttk::wave_sum(i < m ? fma(x, x, 0.0) : 0.0);
      const double alpha = wj[j];
      double tj, sc, beta;
      if (s2 == 0.0) {
        tj = 0.0;
        beta = alpha;
        sc = 0.0;
      } else {
        const double nrm = sqrt(alpha * alpha + s2);
        beta = (alpha >= 0.0) ? -nrm : nrm;
        tj = (beta - alpha) / beta;
        sc = 1.0 / (alpha - beta);
      }
      const double v = x * sc;
      if (tj != 0.0) {
        for (int c = j + 1 + ((wid - (j + 1) % nw + nw) % nw); c < n; c += nw) {
          double *wc = W + (int64_t)c * m;
          const double init = (lane == 0) ? wc[j] : 0.0;
          double d = i < m ? fma(v, wc[i], init) : init;
          d = ttk::wave_sum(d) * tj;
          if (lane == 0) wc[j] -= d;
          if (i < m) wc[i] -= d * v;
        }
      }
      __syncthreads();
      if (wid == j % nw) {  // column j's owner stores the reflector, beta and tau (every wave has read
                            // column j above; nobody reads it again before the loop ends)
        if (i < m) wj[i] = v;
        if (lane == 0) {
          wj[j] = beta;
          tau[j] = tj;
        }
      }
    }
    __syncthreads();
  } else
  for (int j = 0; j < k; ++j) {
    double *wj = W + (int64_t)j * m;
    double s2 = ttk::chain_ahead<CU>(
        ttk::steps_below(j + 1 + tid, m, nt), [&](int q) { return wj[j + 1 + tid + nt * q]; },
        [&](int q) { return wj[j + 1 + tid + nt * q]; }, 0.0);
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
        double d = ttk::chain_ahead<CU>(
            ttk::steps_below(j + 1 + lane, m, 64), [&](int q) { return wj[j + 1 + lane + 64 * q]; },
            [&](int q) { return wc[j + 1 + lane + 64 * q]; }, (lane == 0) ? wc[j] : 0.0);
        d = ttk::wave_sum(d) * tj;
        if (lane == 0) wc[j] -= d;
        ttk::axpy_sub_strided(wc, wj, d, j + 1 + lane, m, 64);
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
  // column c of Q only ever meets the reflectors j <= c, in the order j = c, c-1, ..., 0 -- so each
  // wave takes whole columns through all their reflectors with no block barrier between reflectors
  // (the per-column operations and their order are the reflector-by-reflector loop's: bit-identical;
  // one wave's LDS / global accesses stay in program order behind the workgroup fence)
  for (int c = wid; c < k; c += nw) {
    double *qc = Qc + (int64_t)c * m;
    for (int j = c; j >= 0; --j) {
      const double tj = tau[j];
      if (tj == 0.0) continue;
      const double *v = W + (int64_t)j * m;
      double d = ttk::chain_ahead<CU>(
          ttk::steps_below(j + 1 + lane, m, 64), [&](int q) { return v[j + 1 + lane + 64 * q]; },
          [&](int q) { return qc[j + 1 + lane + 64 * q]; }, (lane == 0) ? qc[j] : 0.0);
      d = ttk::wave_sum(d) * tj;
      if (lane == 0) qc[j] -= d;
      ttk::axpy_sub_strided(qc, v, d, j + 1 + lane, m, 64);
      __threadfence_block();
    }
  }
  __syncthreads();
  if (colmajor) {
    for (int64_t e = tid; e < (int64_t)m * k; e += nt) Q[e] = Qc[e];
    return;
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
  const double abs_floor = EPS * fro;
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

// ------------------------------------------------------------------ extreme eigenpair
// One eigenpair (the smallest, which=0, or the largest, which=1) of a symmetric n x n matrix:
//   1. Householder tridiagonalisation Q^T A Q = T (row-oriented dsytd2; reflector k is kept in
//      row k right of the diagonal, its tau in tv[k]),
//   2. Sturm-count multisection on T: every thread evaluates one shift, so each round shrinks
//      the bracket ~1000x (about 6 rounds reach working precision),
//   3. inverse iteration on T (tridiagonal LU with partial pivoting as dgttrf/dgtts2, thread 0),
//   4. back-transform y = H_0 ... H_{n-3} z by one wave.
// ~4/3 n^3 flops once, against ~10 sweeps x 4 n^3 for cyclic Jacobi; only the extreme pair is
// used on the path (`_min_eigpair` / `_gen_max_eig` in tt_eig.py).
// Phases 2-4 of the extreme eigenpair, shared by the one-workgroup kernel and the finish kernel of
// the multi-workgroup tridiagonalisation: T from the reduced A (reflectors kept in A's rows), Sturm
// multisection, inverse iteration, back-transform.
// RA: the back-transform holds each reflector in registers, loaded one ahead (A in global memory: the
// one-launch-per-step path's tri_finish_kernel); with A in LDS the plain loop is the faster one
// stage (RA only): 2 x BT_RB x 512 doubles of LDS -- the back-transform's reflectors then come from
// LDS, staged BT_RB rows at a time by waves 1..BT_RB while wave 0 applies the previous block
constexpr int BT_RB = 8;
template <bool RA = false>
__device__ __forceinline__ void tridiag_extreme_finish(double *A, int n, int which, double *dv, double *ov, double *ev2, double *tv,
                                       double *z, double *fd, double *fdu, double *fdu2, double *fdl, double *fpiv,
                                       double *__restrict__ ev_out, double *__restrict__ vec_out, int lda,
                                       int timing = 0, double *stage = nullptr) {
  __shared__ double sh_a, sh_b;
  __shared__ int sh_first[2];  // round r's first shift with count >= target, by round parity
  const int tid = threadIdx.x, nt = blockDim.x;
  unsigned long long t_ph = timing ? wall_clock64() : 0;
#define TTK_EPHASE(K)                                   \
  if (timing && tid == 0) {                             \
    const unsigned long long t1 = wall_clock64();       \
    atomicAdd(&g_dbg[K], t1 - t_ph);                    \
    t_ph = t1;                                          \
  }
  const int lane = tid & 63, wid = tid >> 6;
  if (tid == 0) {
    if (n >= 2) {
      dv[n - 2] = A[(int64_t)(n - 2) * lda + n - 2];
      ov[n - 2] = A[(int64_t)(n - 2) * lda + n - 1];
      tv[n - 2] = 0.0;
    }
    dv[n - 1] = A[(int64_t)(n - 1) * lda + n - 1];
  }
  __syncthreads();
  for (int i = tid; i + 1 < n; i += nt) ev2[i] = ov[i] * ov[i];
  __syncthreads();
  // Gershgorin bracket
  double lo = 1e308, hi = -1e308, emax2 = 0.0;
  for (int i = 0; i < n; ++i) {
    const double r = (i > 0 ? fabs(ov[i - 1]) : 0.0) + (i + 1 < n ? fabs(ov[i]) : 0.0);
    lo = fmin(lo, dv[i] - r);
    hi = fmax(hi, dv[i] + r);
    if (i + 1 < n) emax2 = fmax(emax2, ev2[i]);
  }
  const double tnorm = fmax(fmax(fabs(lo), fabs(hi)), 1e-300);
  const double pivmin = fmax(2.2250738585072014e-308 * fmax(emax2, 1.0), 1e-290);
  const double pad = 2.0 * EPS * tnorm + 4.0 * pivmin;
  lo -= pad;
  hi += pad;
  const int target = which ? n : 1;  // smallest x with #{eig < x} >= target
  if (tid == 0) {
    sh_a = lo;
    sh_b = hi;
    sh_first[0] = nt < 256 ? nt : 256;
  }
  __syncthreads();
  // ---- 2. multisection (two barriers per round: the next round's slot is reset with the update)
  // at most 4 waves evaluate shifts: the Sturm recurrence is issue-bound, more waves per SIMD only
  // stretch each round (the extra waves of a 16-wave block wait at the barriers)
  const int ns = nt < 256 ? nt : 256;
  for (int round = 0; round < 16; ++round) {
    const double a = sh_a, b = sh_b;
    if (b - a <= 2.0 * EPS * fmax(fabs(a), fabs(b)) + 2.0 * pivmin) break;
    if (timing == 1 && tid == 0) atomicAdd(&g_dbg[3], 1ull);  // rounds (diagnostics)
    if (tid < ns) {
      const double x = a + (b - a) * (double)(tid + 1) / (double)(ns + 1);
      int cnt = 0;
      double q = dv[0] - x;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
      int i = 1;
      for (; i + 3 < n; i += 4) {  // operands of 4 steps loaded ahead of the recurrence
        const double d0 = dv[i] - x, d1 = dv[i + 1] - x, d2 = dv[i + 2] - x, d3 = dv[i + 3] - x;
        const double e0 = ev2[i - 1], e1 = ev2[i], e2 = ev2[i + 1], e3 = ev2[i + 2];
        q = d0 - e0 * fast_rcp(q);
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
        q = d1 - e1 * fast_rcp(q);
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
        q = d2 - e2 * fast_rcp(q);
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
        q = d3 - e3 * fast_rcp(q);
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
      }
      for (; i < n; ++i) {
        q = dv[i] - x - ev2[i - 1] * fast_rcp(q);
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
      }
      if (cnt >= target) atomicMin(&sh_first[round & 1], tid);
    }
    __syncthreads();
    if (tid == 0) {
      const int f = sh_first[round & 1];
      sh_first[(round + 1) & 1] = ns;
      sh_a = (f == 0) ? a : a + (b - a) * (double)f / (double)(ns + 1);
      sh_b = (f >= ns) ? b : a + (b - a) * (double)(f + 1) / (double)(ns + 1);
    }
    __syncthreads();
  }
  const double lam = 0.5 * (sh_a + sh_b);
  if (timing == 1 && tid == 0) atomicAdd(&g_dbg[2], 1ull);  // calls
  TTK_EPHASE(5)
  // ---- 3. inverse iteration on T (thread 0, O(n) per solve).  The running pivot row, the next
  // diagonal and the solve recurrences are carried in registers; the LDS arrays are written once
  // per element and never read back inside a recurrence (LDS store->load latency would otherwise
  // sit on every step of the serial chain).  Same operations in the same order as dgttrf/dgtts2.
  if (tid == 0) {
    double d = dv[0] - lam;
    double u = (1 < n) ? ov[0] : 0.0;
    // dgttrf step i from l = ov[i], dn = dv[i+1] - lam, un = ov[i+1] (0 past the end).  The loops
    // below load the operands of 4 steps ahead of the recurrence (one LDS round trip per 4 steps).
    auto trf = [&](int i, double l, double dn, double un) {
      double u2 = 0.0, pvt = 0.0, lf = l, dfin = d;
      if (fabs(d) >= fabs(l)) {
        if (d != 0.0) {
          const double f = l * fast_rcp(d);
          lf = f;
          dn -= f * u;
        }
        fdu[i] = u;
      } else {
        const double f = d * fast_rcp(l);
        dfin = l;
        lf = f;
        fdu[i] = dn;
        dn = u - f * dn;
        if (i + 2 < n) {
          u2 = un;
          un = -f * un;
        }
        pvt = 1.0;
      }
      fd[i] = dfin;
      fdl[i] = lf;
      fdu2[i] = u2;
      fpiv[i] = pvt;
      d = dn;
      u = un;
    };
    int i = 0;
    for (; i + 4 < n; i += 4) {
      const double o0 = ov[i], o1 = ov[i + 1], o2 = ov[i + 2], o3 = ov[i + 3], o4 = ov[i + 4];
      const double d1 = dv[i + 1], d2 = dv[i + 2], d3 = dv[i + 3], d4 = dv[i + 4];
      trf(i, o0, d1 - lam, o1);
      trf(i + 1, o1, d2 - lam, o2);
      trf(i + 2, o2, d3 - lam, o3);
      trf(i + 3, o3, d4 - lam, (i + 5 < n) ? o4 : 0.0);
    }
    for (; i + 1 < n; ++i) trf(i, ov[i], dv[i + 1] - lam, (i + 2 < n) ? ov[i + 1] : 0.0);
    fd[n - 1] = d;
    fdu[n - 1] = 0.0;
    fdl[n - 1] = 0.0;
    fdu2[n - 1] = 0.0;
    fpiv[n - 1] = 0.0;
    const double tiny = EPS * tnorm;
    for (int i = 0; i < n; ++i) {  // store 1/U(i,i) for the solves
      double di = fd[i];
      if (fabs(di) < tiny) di = copysign(tiny, di == 0.0 ? 1.0 : di);
      fd[i] = fast_rcp(di);
    }
    uint32_t h = 0x9e3779b9u;  // fixed pseudo-random start (dstein uses a random start)
    for (int i = 0; i < n; ++i) {
      h ^= h << 13;
      h ^= h >> 17;
      h ^= h << 5;
      z[i] = 0.5 + (double)(h & 0xffffff) / 16777216.0;
    }
    double sc = 1.0;  // scale of the previous iterate, applied as it is loaded
    for (int it = 0; it < 3; ++it) {
      double zc = z[0] * sc;
      auto fwd = [&](int i, double zn, double l, double pv_) {  // dgtts2 forward step
        if (pv_ == 0.0) {
          zn -= l * zc;
          z[i] = zc;
          zc = zn;
        } else {
          z[i] = zn;
          zc = zc - l * zn;
        }
      };
      int i = 0;
      for (; i + 4 < n; i += 4) {  // z[i+1..i+4] are loaded before this block writes z[i..i+3]
        const double z1_ = z[i + 1], z2_ = z[i + 2], z3_ = z[i + 3], z4_ = z[i + 4];
        const double l0 = fdl[i], l1 = fdl[i + 1], l2 = fdl[i + 2], l3 = fdl[i + 3];
        const double q0 = fpiv[i], q1 = fpiv[i + 1], q2 = fpiv[i + 2], q3 = fpiv[i + 3];
        fwd(i, z1_ * sc, l0, q0);
        fwd(i + 1, z2_ * sc, l1, q1);
        fwd(i + 2, z3_ * sc, l2, q2);
        fwd(i + 3, z4_ * sc, l3, q3);
      }
      for (; i + 1 < n; ++i) fwd(i, z[i + 1] * sc, fdl[i], fpiv[i]);
      double z1 = zc * fd[n - 1], z2 = 0.0;
      z[n - 1] = z1;
      double mx = fabs(z1);
      if (n > 1) {
        const double zz = (z[n - 2] - fdu[n - 2] * z1) * fd[n - 2];
        z[n - 2] = zz;
        z2 = z1;
        z1 = zz;
        mx = fmax(mx, fabs(zz));
      }
      auto bwd = [&](int i, double zi, double du, double du2, double di) {
        const double zz = (zi - du * z1 - du2 * z2) * di;
        z[i] = zz;
        z2 = z1;
        z1 = zz;
        mx = fmax(mx, fabs(zz));
      };
      int ib = n - 3;
      for (; ib >= 3; ib -= 4) {
        const double a0 = z[ib], a1 = z[ib - 1], a2 = z[ib - 2], a3 = z[ib - 3];
        const double u0 = fdu[ib], u1 = fdu[ib - 1], u2_ = fdu[ib - 2], u3 = fdu[ib - 3];
        const double w0 = fdu2[ib], w1 = fdu2[ib - 1], w2 = fdu2[ib - 2], w3 = fdu2[ib - 3];
        const double e0 = fd[ib], e1 = fd[ib - 1], e2 = fd[ib - 2], e3 = fd[ib - 3];
        bwd(ib, a0, u0, w0, e0);
        bwd(ib - 1, a1, u1, w1, e1);
        bwd(ib - 2, a2, u2_, w2, e2);
        bwd(ib - 3, a3, u3, w3, e3);
      }
      for (; ib >= 0; --ib) bwd(ib, z[ib], fdu[ib], fdu2[ib], fd[ib]);
      sc = mx > 0.0 ? fast_rcp(mx) : 1.0;
    }
    double nn = 0.0;
    for (int i = 0; i < n; ++i) {
      const double t = z[i] * sc;
      z[i] = t;
      nn += t * t;
    }
    const double sc2 = 1.0 / sqrt(nn);
    for (int i = 0; i < n; ++i) z[i] *= sc2;
    ev_out[0] = lam;
  }
  __syncthreads();
  TTK_EPHASE(6)
  // ---- 4. back-transform by wave 0 (no block barriers inside).  Up to 8 elements per lane (n <= 514):
  // each reflector is held in registers, loaded one reflector ahead -- the plain loop below waited
  // one global round trip per reflector for A's row k, then read the row again for the update; the
  // same FMAs in the same order (acc += v z, z -= acc v): bit-identical
  constexpr int BT_VR = 8;
  if (RA && stage && n - 1 <= 64 * BT_VR && n >= 3 && nt >= 64 * (BT_RB + 1)) {
    // the same steps as the register loop below, each reflector read from an LDS block that waves
    // 1..BT_RB filled from global memory while wave 0 worked through the previous block: wave 0's
    // global round trip per reflector becomes one block barrier per BT_RB reflectors.  The values and
    // the FMAs, in their order, are the register loop's (bit-identical)
    const int ktop = n - 3, nblk = (ktop + BT_RB) / BT_RB;
    auto stage_row = [&](int b, int r) {  // row r of block b into its slot (zeros past the reflector)
      const int k = ktop - b * BT_RB - r;
      if (k < 0) return;
      const double *v = A + (int64_t)k * lda + k + 1;
      const int m = n - k - 1;
      double *dst = stage + ((int64_t)(b & 1) * BT_RB + r) * (64 * BT_VR);
#pragma unroll
      for (int u = 0; u < BT_VR; ++u) dst[lane + 64 * u] = lane + 64 * u < m ? v[lane + 64 * u] : 0.0;
    };
    if (wid < BT_RB) stage_row(0, wid);
    __syncthreads();
    for (int b = 0; b < nblk; ++b) {
      if (wid == 0) {
        for (int r = 0; r < BT_RB; ++r) {
          const int k = ktop - b * BT_RB - r;
          if (k < 0) break;
          const double tau = tv[k];
          if (tau != 0.0) {
            const double *vs = stage + ((int64_t)(b & 1) * BT_RB + r) * (64 * BT_VR);
            double vc[BT_VR];
#pragma unroll
            for (int u = 0; u < BT_VR; ++u) vc[u] = vs[lane + 64 * u];
            double *zk = z + k + 1;
            const int m = n - k - 1;
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < BT_VR; ++u)
              if (lane + 64 * u < m) acc = fma(vc[u], zk[lane + 64 * u], acc);
            acc = tau * ttk::wave_sum(acc);
#pragma unroll
            for (int u = 0; u < BT_VR; ++u)
              if (lane + 64 * u < m) zk[lane + 64 * u] = fma(-acc, vc[u], zk[lane + 64 * u]);
            __threadfence_block();
          }
        }
      } else if (wid <= BT_RB && b + 1 < nblk) {
        stage_row(b + 1, wid - 1);
      }
      __syncthreads();
    }
  } else if (RA && wid == 0 && n - 1 <= 64 * BT_VR && n >= 3) {
    double vc[BT_VR], vn[BT_VR];
    auto load_row = [&](int k, double *dst) {
      const double *v = A + (int64_t)k * lda + k + 1;
      const int m = n - k - 1;
#pragma unroll
      for (int u = 0; u < BT_VR; ++u) dst[u] = lane + 64 * u < m ? v[lane + 64 * u] : 0.0;
    };
    load_row(n - 3, vc);
    for (int k = n - 3; k >= 0; --k) {
      if (k > 0) load_row(k - 1, vn);
      const double tau = tv[k];
      if (tau != 0.0) {
        double *zk = z + k + 1;
        const int m = n - k - 1;
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < BT_VR; ++u)
          if (lane + 64 * u < m) acc = fma(vc[u], zk[lane + 64 * u], acc);
        acc = tau * ttk::wave_sum(acc);
#pragma unroll
        for (int u = 0; u < BT_VR; ++u)
          if (lane + 64 * u < m) zk[lane + 64 * u] = fma(-acc, vc[u], zk[lane + 64 * u]);
        __threadfence_block();
      }
#pragma unroll
      for (int u = 0; u < BT_VR; ++u) vc[u] = vn[u];
    }
  } else if (wid == 0) {
    for (int k = n - 3; k >= 0; --k) {
      const double tau = tv[k];
      if (tau == 0.0) continue;
      const double *v = A + (int64_t)k * lda + k + 1;
      double *zk = z + k + 1;
      const int m = n - k - 1;
      double acc = 0.0;
      for (int j = lane; j < m; j += 64) acc += v[j] * zk[j];
      acc = tau * ttk::wave_sum(acc);
      for (int j = lane; j < m; j += 64) zk[j] -= acc * v[j];
      __threadfence_block();
    }
  }
  __syncthreads();
  TTK_EPHASE(7)
#undef TTK_EPHASE
  for (int i = tid; i < n; i += nt) vec_out[i] = z[i];
}

int64_t syev_extreme_need(int n) { return (int64_t)n * n + 13 * (int64_t)n + 32; }

__global__ __launch_bounds__(1024) void syev_extreme_kernel(const double *__restrict__ Ain, int n, int which,
                                                            double *__restrict__ ev_out,
                                                            double *__restrict__ vec_out,
                                                            double *__restrict__ gwork, int use_lds) {
  extern __shared__ double lds[];
  double *A = use_lds ? lds : gwork;
  double *dv = A + (int64_t)n * n;  // diag(T)
  double *ov = dv + n;              // offdiag(T)
  double *ev2 = ov + n;             // offdiag^2
  double *tv = ev2 + n;             // tau per reflector
  double *pv = tv + n;              // matvec scratch
  double *z = pv + n;               // eigenvector (T basis, then A basis)
  double *fd = z + n, *fdu = fd + n, *fdu2 = fdu + n, *fdl = fdu2 + n, *fpiv = fdl + n;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  for (int e = tid; e < n * n; e += nt) A[e] = Ain[e];
  __syncthreads();
  // ---- 1. tridiagonalisation (3 barriers per reflector)
  for (int k = 0; k + 2 < n; ++k) {
    double *v = A + (int64_t)k * n + k + 1;  // x = A[k, k+1:], becomes the reflector
    const int m = n - k - 1;
    if (wid == 0) {  // reflector by wave 0
      double part = 0.0;
      #pragma unroll 8
      for (int i = 1 + lane; i < m; i += 64) part += v[i] * v[i];
      const double sigma = ttk::wave_sum(part);
      const double alpha = v[0];
      double tau = 0.0, beta = alpha;
      if (sigma > 0.0) {
        beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
        tau = (beta - alpha) / beta;
        const double sc = 1.0 / (alpha - beta);
        #pragma unroll 8
        for (int i = 1 + lane; i < m; i += 64) v[i] *= sc;
      }
      if (lane == 0) {
        v[0] = 1.0;
        tv[k] = tau;
        ov[k] = beta;
        dv[k] = A[(int64_t)k * n + k];
      }
    }
    __syncthreads();
    const double tau = tv[k];
    if (tau == 0.0) continue;
    // p = tau * A22 v with g lanes per row
    int g = 1;
    while (g < 16 && 2 * g * m <= nt) g *= 2;
    const int gl = tid & (g - 1), ng = nt / g;
    for (int i = tid / g; i < m; i += ng) {
      const double *ai = A + (int64_t)(k + 1 + i) * n + k + 1;
      double acc = 0.0;
      for (int j = gl; j < m; j += g) acc += ai[j] * v[j];
      acc = ttk::group_sum_rt(acc, g);
      if (gl == 0) pv[i] = tau * acc;
    }
    __syncthreads();
    double part = 0.0;  // every wave forms K = tau/2 p^T v itself (no barrier)
    #pragma unroll 8
    for (int i = lane; i < m; i += 64) part += pv[i] * v[i];
    const double K = 0.5 * tau * ttk::wave_sum(part);
    for (int i = wid; i < m; i += nw) {  // A22 -= v w^T + w v^T, w = p - K v
      const double vi = v[i], wi = pv[i] - K * vi;
      double *ai = A + (int64_t)(k + 1 + i) * n + k + 1;
      for (int j = lane; j < m; j += 64) {
        const double vj = v[j];
        ai[j] -= vi * (pv[j] - K * vj) + wi * vj;
      }
    }
    __syncthreads();
  }
  tridiag_extreme_finish(A, n, which, dv, ov, ev2, tv, z, fd, fdu, fdu2, fdl, fpiv, ev_out, vec_out, n);
}

// Small-n extreme eigenpair (n <= SYEV_SMALL_N), built for latency: 4 waves, A in LDS with an odd
// leading dimension (row starts on different banks), 2 barriers per reflector.
//   reflector  wave 0 (dlarfg on row k, which holds the sub-column by symmetry)
//   p = tau A22 v   two lanes per row (row i -> lanes 2i, 2i+1 of one wave), halves combined by a
//                   lane-pair shuffle; v read as LDS broadcasts
//   K = tau/2 p^T v every wave redundantly (no barrier); w = p - K v kept in registers per column
//   A22 -= v w^T + w v^T   one wave per row, lanes over columns (<= 2 per lane), A touched once
// Same reflector convention (LAPACK dlarfg) and finish (Sturm multisection + inverse iteration) as
// syev_extreme_kernel, so both paths produce the same eigenpair to rounding.
constexpr int SYEV_SMALL_N = 128;

// the rank-2 update A22 -= v w^T + w v^T of syev_small_kernel, rows i = wid, wid + NW, ...: A22's rows,
// the reflector v (row k of A, left of A22's rows) and p never overlap -- said so, a wave's next rows'
// loads issue ahead of this row's stores (possible aliasing had each row wait for the previous row's
// LDS stores).  The same operations per element: bit-identical.
template <int NW>
__device__ __forceinline__ void syev_rank2_rows(double *__restrict__ A22, int ld, const double *__restrict__ v,
                                                const double *__restrict__ pv, int m, int wid, double K, int j0,
                                                int j1, double v0, double v1, double w0, double w1) {
#pragma unroll 4
  for (int i = wid; i < m; i += NW) {
    const double vi = v[i], wi = fma(-K, vi, pv[i]);
    double *ai = A22 + i * ld;
    if (j0 < m) ai[j0] -= fma(vi, w0, wi * v0);
    if (j1 < m) ai[j1] -= fma(vi, w1, wi * v1);
  }
}

// the same for rows first, first + S, ... (S wave-uniform; syev_small_kernel gives wave 0 row 0 alone
// and the other waves the rest), in batches of B rows whose operands are loaded before any of their
// stores.  Rows past m load row m - 1, lanes past m load column 0, and those lanes store into a
// scratch slot (`dummy`, 32 doubles nobody reads), so a batch has no branches.  The same operations
// per stored element: bit-identical.
template <int B>
__device__ __forceinline__ void syev_rank2_rows_b(double *__restrict__ A22, int ld, const double *__restrict__ v,
                                                  const double *__restrict__ pv, int m, int first, int S, double K,
                                                  int j0, int j1, double v0, double v1, double w0, double w1,
                                                  double *__restrict__ dummy) {
  // wide (m > 64): j0 < m on every lane, and column j0 + 64 past m still lies inside the LDS block
  // (the next row, or the arrays after A), so x1 is read unguarded -- one ds_read2 with x0
  const bool c0 = j0 < m, c1 = j1 < m, wide = m > 64;
  const int l0 = c0 ? j0 : 0;
  double *const d = dummy + (j0 & 31);
  for (int i0 = first; i0 < m; i0 += S * B) {
    double vi[B], pi[B], x0[B], x1[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int i = min(i0 + b * S, m - 1);
      const double *ai = A22 + i * ld;
      vi[b] = v[i];
      pi[b] = pv[i];
      x0[b] = ai[l0];
      x1[b] = wide ? ai[l0 + 64] : 0.0;
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int i = i0 + b * S;
      const bool ok = i < m;
      const double wi = fma(-K, vi[b], pi[b]);
      double *ai = A22 + (ok ? i : 0) * ld;
      *(ok && c0 ? ai + j0 : d) = x0[b] - fma(vi[b], w0, wi * v0);
      if (wide) *(ok && c1 ? ai + j1 : d) = x1[b] - fma(vi[b], w1, wi * v1);
    }
  }
}

// GG: lanes per row in the symv (NT / 128 by default: rows <= 127); <512, 2> keeps the 4-wave kernel's
// symv (2 lanes per row, rows <= 255) and spreads only the rank-2 rows over 8 waves -- every value the
// same expression in the same order as <256> (bit-identical; TTK_KNOB_SYEV_WAVES8 selects it)
template <int NT, int GG = NT / 128>
__global__ __launch_bounds__(NT) void syev_small_kernel(const double *__restrict__ Ain, int n, int which,
                                                        double *__restrict__ ev_out, double *__restrict__ vec_out,
                                                        int timing, int var) {
  constexpr int NW = NT / 64, G = GG;  // waves; lanes per row in the symv
  extern __shared__ double lds[];
  const int ld = n | 1;
  double *A = lds;
  double *dv = A + (int64_t)n * ld, *ov = dv + n, *ev2 = ov + n, *tv = ev2 + n, *pv = tv + n, *z = pv + n;
  double *fd = z + n, *fdu = fd + n, *fdu2 = fdu + n, *fdl = fdu2 + n, *fpiv = fdl + n;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const unsigned long long t_ph0 = timing ? wall_clock64() : 0;
  for (int e = tid; e < n * n; e += NT) {
    const int i = e / n, j = e - i * n;
    A[i * ld + j] = Ain[e];
  }
  __syncthreads();
  // two barriers per reflector: wave 0 owns A22's first row in the rank-2 update, so right after
  // updating it (same wave, LDS order) it builds the next reflector from that row while the other
  // waves finish their rows; nobody else reads the row in that phase.  `var` (TTK_SYEV_VAR, A/B
  // timing; every setting bit-identical): 4 = the symv's lane-group sums by DPP instead of LDS
  // permutes, 8 (4 waves) / 16 (16 waves) = wave 0 updates row 0 only (it was the last to reach the
  // step's second barrier: its share of the rows plus the reflector), the other waves the remaining
  // rows -- n = 40 134.7 -> 126.2 us with 4 waves, slower with 16 (r05_syev_small.txt).
  auto reflector = [&](int k) {  // wave 0: dlarfg on row k (the sub-column by symmetry)
    double *v = A + k * ld + k + 1;
    const int m = n - k - 1;
    const double x1 = (1 + lane < m) ? v[1 + lane] : 0.0;
    const double x2 = (65 + lane < m) ? v[65 + lane] : 0.0;
    const double sigma = ttk::wave_sum(fma(x1, x1, x2 * x2));
    const double alpha = v[0];
    double tau = 0.0, beta = alpha;
    if (sigma > 0.0) {
      beta = -copysign(sqrt(fma(alpha, alpha, sigma)), alpha);
      tau = (beta - alpha) / beta;
      const double sc = 1.0 / (alpha - beta);
      if (1 + lane < m) v[1 + lane] = x1 * sc;
      if (65 + lane < m) v[65 + lane] = x2 * sc;
    }
    if (lane == 0) {
      v[0] = 1.0;
      tv[k] = tau;
      ov[k] = beta;
      dv[k] = A[k * ld + k];
    }
  };
  if (wid == 0 && n > 2) reflector(0);
  __syncthreads();
  // timing == 2: wave 0's cycles per step phase into the debug counters 0..5 (symv, barrier, K,
  // rank-2 rows, reflector, barrier) -- diagnostics only, the stamps wait on outstanding LDS ops
  unsigned long long t_s = timing == 2 ? clock64() : 0;
#define TTK_SSTAMP(K)                                       \
  if (timing == 2 && wid == 0) {                            \
    const unsigned long long t1 = clock64();                \
    if (lane == 0) atomicAdd(&g_dbg[K], t1 - t_s);          \
    t_s = t1;                                               \
  }
  for (int k = 0; k + 2 < n; ++k) {
    const double *v = A + k * ld + k + 1;
    const int m = n - k - 1;
    const double tau = tv[k];
    if (tau != 0.0) {
      const double *A22 = A + (k + 1) * ld + k + 1;
      {  // p = tau A22 v: row r = tid / G, lane h = tid % G of the row takes columns h, h+G, ...
        const int r = tid / G, h = tid % G;
        double acc = 0.0;
        if (r < m) {  // four independent chains: the LDS loads of one batch overlap
          const double *ar = A22 + r * ld;
          double a1 = 0.0, a2 = 0.0, a3 = 0.0;
          int j = h;
          for (; j + 3 * G < m; j += 4 * G) {
            acc = fma(ar[j], v[j], acc);
            a1 = fma(ar[j + G], v[j + G], a1);
            a2 = fma(ar[j + 2 * G], v[j + 2 * G], a2);
            a3 = fma(ar[j + 3 * G], v[j + 3 * G], a3);
          }
          for (; j < m; j += G) acc = fma(ar[j], v[j], acc);
          acc = (acc + a1) + (a2 + a3);
        }
        if (var & 4) {  // DPP: the xor-butterfly's sums (both lanes of a pair hold a + b), no LDS permutes
          acc = ttk::group_sum<G>(acc);
        } else {
#pragma unroll
          for (int o = 1; o < G; o <<= 1) acc += __shfl_xor(acc, o, 64);
        }
        if (h == 0 && r < m) pv[r] = tau * acc;
      }
      TTK_SSTAMP(0)
      __syncthreads();
      TTK_SSTAMP(1)
      const int j0 = lane, j1 = lane + 64;
      const double v0 = j0 < m ? v[j0] : 0.0, v1 = j1 < m ? v[j1] : 0.0;
      const double p0 = j0 < m ? pv[j0] : 0.0, p1 = j1 < m ? pv[j1] : 0.0;
      const double K = 0.5 * tau * ttk::wave_sum(fma(p0, v0, p1 * v1));
      const double w0 = fma(-K, v0, p0), w1 = fma(-K, v1, p1);
      TTK_SSTAMP(2)
      if (var & (NT <= 512 ? 8 : 16)) {  // wave 0 updates row 0 only, then the next reflector
        if (wid == 0)
          syev_rank2_rows_b<1>(A + (k + 1) * ld + k + 1, ld, v, pv, m, 0, m, K, j0, j1, v0, v1, w0, w1, fpiv + n);
        else
          syev_rank2_rows_b<4>(A + (k + 1) * ld + k + 1, ld, v, pv, m, wid, NW - 1, K, j0, j1, v0, v1, w0, w1,
                               fpiv + n);
      } else
        syev_rank2_rows<NW>(A + (k + 1) * ld + k + 1, ld, v, pv, m, wid, K, j0, j1, v0, v1, w0, w1);
      TTK_SSTAMP(3)
    }
    if (wid == 0 && k + 3 < n) {
      __threadfence_block();
      reflector(k + 1);
    }
    TTK_SSTAMP(4)
    __syncthreads();
    TTK_SSTAMP(5)
  }
#undef TTK_SSTAMP
  if (timing == 1 && tid == 0) atomicAdd(&g_dbg[4], wall_clock64() - t_ph0);
  tridiag_extreme_finish(A, n, which, dv, ov, ev2, tv, z, fd, fdu, fdu2, fdl, fpiv, ev_out, vec_out, ld, timing == 1);
}

int64_t syev_small_need(int n) { return (int64_t)n * (n | 1) + 13 * (int64_t)n + 32; }

// Multi-workgroup Householder tridiagonalisation for n beyond LDS: per reflector k two launches over
// row blocks of TRB rows, (1) rank-2 update of step k-1 on the block's rows, then the block owning
// row k builds reflector k; (2) p = tau A22 v on the block's rows and the block's part of p^T v.
// A is n x n row-major in global scratch; the reflectors stay in A's rows as in the LDS kernel.
constexpr int TRB = 16;

__global__ __launch_bounds__(256) void tri_update_kernel(double *A, int n, int k, double *tv, double *ov, double *dv,
                                                         const double *pv, const double *partials, int nblk) {
  __shared__ double red[16];
  __shared__ double sK;
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  const int r0 = blockIdx.x * TRB, r1 = r0 + TRB < n ? r0 + TRB : n;
  const int kp = k - 1;
  if (kp >= 0 && r1 > kp + 1) {
    const double taup = tv[kp];
    if (taup != 0.0) {
      if (wid == 0) {
        double acc = 0.0;
        for (int i = lane; i < nblk; i += 64) acc += partials[i];
        acc = ttk::wave_sum(acc);
        if (lane == 0) sK = 0.5 * taup * acc;
      }
      __syncthreads();
      const double K = sK;
      const double *v = A + (int64_t)kp * n + kp + 1;
      const int m = n - kp - 1;
      const int rs = r0 > kp + 1 ? r0 : kp + 1;
      for (int r = rs + wid; r < r1; r += nw) {
        const int i = r - kp - 1;
        const double vi = v[i], wi = pv[i] - K * vi;
        double *ar = A + (int64_t)r * n + kp + 1;
#pragma unroll 8
        for (int j = lane; j < m; j += 64) {
          const double vj = v[j];
          ar[j] -= vi * (pv[j] - K * vj) + wi * vj;
        }
      }
    }
  }
  if (k + 2 < n && k >= r0 && k < r1) {  // reflector k (dlarfg) from row k
    __syncthreads();
    double *x = A + (int64_t)k * n + k + 1;
    const int m = n - k - 1;
    double part = 0.0;
    for (int i = 1 + tid; i < m; i += nt) part += x[i] * x[i];
    const double sigma = ttk::block_sum(part, red);
    const double alpha = x[0];
    double tau = 0.0, beta = alpha;
    if (sigma > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
      tau = (beta - alpha) / beta;
      const double sc = 1.0 / (alpha - beta);
      for (int i = 1 + tid; i < m; i += nt) x[i] *= sc;
    }
    __syncthreads();
    if (tid == 0) {
      x[0] = 1.0;
      tv[k] = tau;
      ov[k] = beta;
      dv[k] = A[(int64_t)k * n + k];
    }
  }
}

__global__ __launch_bounds__(256) void tri_matvec_kernel(const double *__restrict__ A, int n, int k,
                                                         const double *__restrict__ tv, double *__restrict__ pv,
                                                         double *__restrict__ partials) {
  __shared__ double red[16];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * TRB, r1 = r0 + TRB < n ? r0 + TRB : n;
  const double tau = tv[k];
  const int m = n - k - 1;
  const double *v = A + (int64_t)k * n + k + 1;
  constexpr int G = 256 / TRB;  // lanes per row
  const int gl = tid & (G - 1), rr = tid / G;
  const int r = r0 + rr;
  double contrib = 0.0;
  if (tau != 0.0 && r < r1 && r >= k + 1) {
    const double *ar = A + (int64_t)r * n + k + 1;
    double acc = 0.0;
#pragma unroll 8
    for (int j = gl; j < m; j += G) acc += ar[j] * v[j];
    acc = ttk::group_sum<G>(acc);
    const int i = r - k - 1;
    if (gl == 0) {
      pv[i] = tau * acc;
      contrib = tau * acc * v[i];
    }
  }
  contrib = ttk::block_sum(contrib, red);
  if (tid == 0) partials[blockIdx.x] = contrib;
}

// lds != 0: the finish's ten length-n vectors live in dynamic LDS (dv, ov, tv staged from gv first), so
// the serial chains of the multisection, the inverse iteration and the back-transform wait on LDS,
// not on L2 round trips; same operations in the same order either way
__global__ __launch_bounds__(1024) void tri_finish_kernel(double *A, int n, int which, double *gv, double *ev_out,
                                                          double *vec_out, int lds) {
  extern __shared__ double fl[];
  double *dv = gv, *ov = dv + n, *ev2 = ov + n, *tv = ev2 + n, *z = tv + n;
  double *fd = z + n, *fdu = fd + n, *fdu2 = fdu + n, *fdl = fdu2 + n, *fpiv = fdl + n;
  if (lds) {
    double *ldv = fl, *lov = ldv + n, *lev2 = lov + n, *ltv = lev2 + n, *lz = ltv + n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      ldv[i] = dv[i];
      lov[i] = ov[i];
      ltv[i] = tv[i];
    }
    __syncthreads();
    tridiag_extreme_finish<true>(A, n, which, ldv, lov, lev2, ltv, lz, lz + n, lz + 2 * n, lz + 3 * n, lz + 4 * n,
                           lz + 5 * n, ev_out, vec_out, n, 0, lds == 2 ? fl + 10 * n : nullptr);
    return;
  }
  tridiag_extreme_finish<true>(A, n, which, dv, ov, ev2, tv, z, fd, fdu, fdu2, fdl, fpiv, ev_out, vec_out, n);
}

// TTK_KNOB_BT_STAGE (default 1): the back-transform's reflectors staged through LDS (lds = 2, n <= 513);
// 0: held in registers, loaded one ahead (bit-identical either way)
static int tri_finish_launch(hipStream_t st, double *A, int n, int which, double *gv, double *ev, double *vec) {
  const bool stg = ttk::ctx().knob[TTK_KNOB_BT_STAGE] && n - 1 <= 512;
  const size_t shm = (10 * (size_t)n + (stg ? 2 * (size_t)BT_RB * 512 : 0)) * sizeof(double);
  const int lds = shm <= 150000 ? (stg ? 2 : 1) : 0;
  if (lds && shm > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(tri_finish_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL(tri_finish_kernel, dim3(1), dim3(1024), lds ? shm : 0, st, A, n, which, gv, ev, vec, lds);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

// One launch per Householder step (replaces tri_update + tri_matvec): every block rebuilds row k
// with the pending rank-2 update of step k-1 and reflector k in LDS (redundantly: no extra launch
// or grid sync), then updates its own rows and forms their part of p = tau A22 v.  The only
// cross-block dependency per step is p itself, carried to the next launch in double-buffered
// global vectors; reflector k reaches A's row k one launch later, when no block reads that row.
constexpr int TRI_FUSED_MAX = 2048;

__global__ __launch_bounds__(256) void tri_step_kernel(double *A, int n, int k, double *tv, double *ov, double *dv,
                                                       double *pvb, double *partb, double *vbuf, int nblk, int rb) {
  __shared__ double xs[TRI_FUSED_MAX + 1];
  __shared__ double red[16];
  __shared__ double s_k, s_tau;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r0 = blockIdx.x * rb, r1 = r0 + rb < n ? r0 + rb : n;
  const int kp = k - 1;
  const double *pvp = pvb + (kp & 1) * (int64_t)n, *ptp = partb + (kp & 1) * (int64_t)nblk;
  const double *vp = vbuf + (kp & 1) * (int64_t)n;  // reflector k-1, relative index (vp[0] = 1)
  double *pvc = pvb + (k & 1) * (int64_t)n, *ptc = partb + (k & 1) * (int64_t)nblk, *vc = vbuf + (k & 1) * (int64_t)n;
  const double taup = kp >= 0 ? tv[kp] : 0.0;
  if (wid == 0) {
    double acc = 0.0;
    if (taup != 0.0)
      for (int i = lane; i < nblk; i += 64) acc += ptp[i];
    acc = ttk::wave_sum(acc);
    if (lane == 0) s_k = 0.5 * taup * acc;
  }
  __syncthreads();
  const double K = s_k;
  // reflector k of the pending-updated row k (relative index jj = j - kp - 1 into step k-1's vectors)
  const int m = n - k - 1;
  {
    const double wk = taup != 0.0 ? pvp[0] - K * vp[0] : 0.0, vk = taup != 0.0 ? vp[0] : 0.0;
    const double *ak = A + (int64_t)k * n;
    for (int j = k + tid; j < n; j += 256) {
      double a = ak[j];
      if (taup != 0.0) {
        const int jj = j - kp - 1;
        const double vj = vp[jj];
        a -= vk * (pvp[jj] - K * vj) + wk * vj;
      }
      xs[j - k] = a;
    }
  }
  __syncthreads();
  double part = 0.0;
  for (int i = 2 + tid; i <= m; i += 256) part += xs[i] * xs[i];
  const double sigma = ttk::block_sum(part, red);
  const double alpha = xs[1];
  double tau = 0.0, beta = alpha;
  if (sigma > 0.0) {
    beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
    tau = (beta - alpha) / beta;
  }
  const double sc = sigma > 0.0 ? 1.0 / (alpha - beta) : 1.0;
  const bool owner_k = k >= r0 && k < r1;
  if (tid == 0) s_tau = tau;
  __syncthreads();  // every thread has read xs[1] / the sigma partials
  for (int i = 1 + tid; i <= m; i += 256) {
    const double v = (i == 1) ? 1.0 : xs[i] * sc;
    xs[i] = v;  // xs[1 + jj] = v_k[jj]
    if (owner_k) vc[i - 1] = v;
  }
  if (owner_k && tid == 0) {
    tv[k] = tau;
    ov[k] = beta;
    dv[k] = xs[0];
  }
  // reflector k-1 into A's row k-1 (nobody reads that row in this launch)
  if (kp >= 0 && kp >= r0 && kp < r1)
    for (int j = kp + 1 + tid; j < n; j += 256) A[(int64_t)kp * n + j] = vp[j - kp - 1];
  __syncthreads();
  // own rows r > k: pending update of step k-1, then p_r = tau <A[r, k+1:], v_k>
  const int rs = r0 > k + 1 ? r0 : k + 1;
  double contrib = 0.0;
  for (int r = rs + wid; r < r1; r += 4) {
    double *ar = A + (int64_t)r * n;
    const int ir = r - kp - 1;
    const double vi = taup != 0.0 ? vp[ir] : 0.0, wi = taup != 0.0 ? pvp[ir] - K * vi : 0.0;
    double acc = 0.0;
    for (int j = k + 1 + lane; j < n; j += 64) {
      double a = ar[j];
      if (taup != 0.0) {
        const int jj = j - kp - 1;
        const double vj = vp[jj];
        a -= vi * (pvp[jj] - K * vj) + wi * vj;
        ar[j] = a;
      }
      acc = fma(a, xs[j - k], acc);
    }
    acc = ttk::wave_sum(acc);
    if (lane == 0) {
      const double pr = tau * acc;
      pvc[r - k - 1] = pr;
      contrib += pr * xs[r - k];
    }
  }
  contrib = ttk::block_sum(contrib, red);
  if (tid == 0) ptc[blockIdx.x] = contrib;
  (void)s_tau;
}

// tri_step_kernel with every global load of the step issued up front into registers (the previous
// step's partials, pivot row k, reflector k-1 and its p vector, the wave's own row): the loads do not
// depend on each other, so a step waits for ONE round of L2 latency instead of three (partials ->
// pivot row -> own row).  The arithmetic, its order and every stored value are tri_step_kernel's
// at rb = 4 (bit-identical; TTK_KNOB_TRI_HOIST = 0 switches back).  NX * 256 >= n - k,
// NP * 64 >= nblk, NR * 64 >= n - k - 1.
// global accesses of a tridiagonalisation step: plain (one launch per step, the kernel boundary
// orders the steps) or sc1 (tri_persist_kernel: the steps of one launch hand their words over)
template <bool SC>
__device__ __forceinline__ double gld(const double *p) {
  if constexpr (SC) return ttk::ld_sc1(p);
  else return *p;
}
template <bool SC>
__device__ __forceinline__ void gst(double *p, double v) {
  if constexpr (SC) ttk::st_sc1(p, v);
  else *p = v;
}

template <int NX, int NP, int NR, bool SC>
__device__ __forceinline__ void tri_hoist_step(double *A, int n, int k, double *tv, double *ov, double *dv,
                                               double *pvb, double *partb, double *vbuf, int nblk, int blk,
                                               double *xs, double *red, double &s_k) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r0 = blk * 4, r1 = r0 + 4 < n ? r0 + 4 : n;
  const int kp = k - 1;
  const double *pvp = pvb + (kp & 1) * (int64_t)n, *ptp = partb + (kp & 1) * (int64_t)nblk;
  const double *vp = vbuf + (kp & 1) * (int64_t)n;  // reflector k-1, relative index (vp[0] = 1)
  double *pvc = pvb + (k & 1) * (int64_t)n, *ptc = partb + (k & 1) * (int64_t)nblk, *vc = vbuf + (k & 1) * (int64_t)n;
  const int m = n - k - 1;
  // ---- loads (values of buffers step k-1 did not write are read but never used: taup == 0 then)
  const double taup = kp >= 0 ? gld<SC>(tv + kp) : 0.0;
  double pa[NP];
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int i = lane + 64 * u;
    pa[u] = (wid == 0 && i < nblk) ? gld<SC>(ptp + i) : 0.0;
  }
  const double v0 = gld<SC>(vp), p0 = gld<SC>(pvp);
  double xa[NX], xv[NX], xp[NX];
#pragma unroll
  for (int u = 0; u < NX; ++u) {
    const int j = k + tid + 256 * u, jj = j - kp - 1;
    const bool ok = j < n;
    xa[u] = ok ? gld<SC>(A + (int64_t)k * n + j) : 0.0;
    xv[u] = ok ? gld<SC>(vp + jj) : 0.0;
    xp[u] = ok ? gld<SC>(pvp + jj) : 0.0;
  }
  const int rs = r0 > k + 1 ? r0 : k + 1;
  const int r = rs + wid;  // this wave's own row (rb = 4: at most one per wave)
  const bool has_row = r < r1;
  double ra[NR], rv[NR], rp[NR], vi = 0.0, pi = 0.0;
  if (has_row) {
    const int ir = r - kp - 1;
    vi = gld<SC>(vp + ir);
    pi = gld<SC>(pvp + ir);
    const double *ar = A + (int64_t)r * n;
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int j = k + 1 + lane + 64 * u, jj = j - kp - 1;
      const bool ok = j < n;
      ra[u] = ok ? gld<SC>(ar + j) : 0.0;
      rv[u] = ok ? gld<SC>(vp + jj) : 0.0;
      rp[u] = ok ? gld<SC>(pvp + jj) : 0.0;
    }
  }
  // ---- the step (tri_step_kernel's operations)
  if (wid == 0) {
    double acc = 0.0;
    if (taup != 0.0) {
#pragma unroll
      for (int u = 0; u < NP; ++u)
        if (lane + 64 * u < nblk) acc += pa[u];
    }
    acc = ttk::wave_sum(acc);
    if (lane == 0) s_k = 0.5 * taup * acc;
  }
  __syncthreads();
  const double K = s_k;
  {
    const double wk = taup != 0.0 ? p0 - K * v0 : 0.0, vk = taup != 0.0 ? v0 : 0.0;
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int j = k + tid + 256 * u;
      if (j < n) {
        double a = xa[u];
        // tri_step_kernel's contraction of a -= vk * (p - K v) + wk * v, spelled out (the compiler
        // contracts the expression differently in this kernel)
        if (taup != 0.0) a -= fma(wk, xv[u], vk * fma(-K, xv[u], xp[u]));
        xs[j - k] = a;
      }
    }
  }
  __syncthreads();
  double part = 0.0;
  for (int i = 2 + tid; i <= m; i += 256) part += xs[i] * xs[i];
  const double sigma = ttk::block_sum(part, red);
  const double alpha = xs[1];
  double tau = 0.0, beta = alpha;
  if (sigma > 0.0) {
    beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
    tau = (beta - alpha) / beta;
  }
  const double sc = sigma > 0.0 ? 1.0 / (alpha - beta) : 1.0;
  const bool owner_k = k >= r0 && k < r1;
  __syncthreads();  // every thread has read xs[1] / the sigma partials
  for (int i = 1 + tid; i <= m; i += 256) {
    const double v = (i == 1) ? 1.0 : xs[i] * sc;
    xs[i] = v;
    if (owner_k) gst<SC>(vc + i - 1, v);
  }
  if (owner_k && tid == 0) {
    gst<SC>(tv + k, tau);
    gst<SC>(ov + k, beta);
    gst<SC>(dv + k, xs[0]);
  }
  if (kp >= 0 && kp >= r0 && kp < r1) {  // reflector k-1 into A's row k-1: the values loaded above
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int j = k + tid + 256 * u;
      if (j < n) gst<SC>(A + (int64_t)kp * n + j, xv[u]);
    }
  }
  __syncthreads();
  double contrib = 0.0;
  if (has_row) {
    double *ar = A + (int64_t)r * n;
    const double wi = taup != 0.0 ? pi - K * vi : 0.0, vv = taup != 0.0 ? vi : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int j = k + 1 + lane + 64 * u;
      if (j < n) {
        double a = ra[u];
        if (taup != 0.0) {
          a -= fma(wi, rv[u], vv * fma(-K, rv[u], rp[u]));  // tri_step_kernel's contraction
          gst<SC>(ar + j, a);
        }
        acc = fma(a, xs[j - k], acc);
      }
    }
    acc = ttk::wave_sum(acc);
    if (lane == 0) {
      const double pr = tau * acc;
      gst<SC>(pvc + r - k - 1, pr);
      contrib += pr * xs[r - k];
    }
  }
  contrib = ttk::block_sum(contrib, red);
  if (tid == 0) gst<SC>(ptc + blk, contrib);
}


template <int NX, int NP, int NR>
__global__ __launch_bounds__(256) void tri_step_hoist_kernel(double *A, int n, int k, double *tv, double *ov,
                                                             double *dv, double *pvb, double *partb, double *vbuf,
                                                             int nblk) {
  __shared__ double xs[NX * 256 + 1];
  __shared__ double red[16];
  __shared__ double s_k;
  tri_hoist_step<NX, NP, NR, false>(A, n, k, tv, ov, dv, pvb, partb, vbuf, nblk, blockIdx.x, xs, red, s_k);
}

// Every step of tri_step_hoist_kernel in ONE launch (TTK_KNOB_TRI_PERSIST): the nblk workgroups stay
// resident and run the steps in turn, each step's global words handed to the next step inside the
// launch (ttk_common.h: sc1 stores, dep_arrive = drain + barrier + agent-scope release + one counter
// add per workgroup; dep_wait = poll until all nblk workgroups arrived from step k-1, then acquire) --
// step k reads only what step k-1 wrote (double-buffered by step parity, as the per-step launches),
// and a workgroup writes step k's words only after every workgroup has finished step k-1, so the
// launch boundary between steps becomes one counter.  The step itself is tri_hoist_step, the same
// source as the per-step kernel: bit-identical (tools/dump_kernels.py, test_gpu_kernels.py).  Roles by
// start ticket; nblk = n / 4 <= 128 workgroups of 256 threads, well inside the chip's resident capacity;
// a wait past DEP_SPIN_MAX is counted (ttk_dep_timeouts) instead of hanging.
template <int NX, int NP, int NR>
__global__ __launch_bounds__(256) void tri_persist_kernel(double *A, int n, double *tv, double *ov, double *dv,
                                                          double *pvb, double *partb, double *vbuf, int nblk,
                                                          unsigned *dep, unsigned target, unsigned tick_base) {
  __shared__ double xs[NX * 256 + 1];
  __shared__ double red[16];
  __shared__ double s_k;
  const int blk = ttk::ticket(dep, tick_base);
  for (int k = 0; k + 2 < n; ++k) {
    if (k > 0) ttk::dep_wait(dep, target + (unsigned)nblk * (unsigned)k);
    tri_hoist_step<NX, NP, NR, true>(A, n, k, tv, ov, dv, pvb, partb, vbuf, nblk, blk, xs, red, s_k);
    ttk::dep_arrive(dep);
  }
}

// after the last step (k = n-3): pending update of step n-3 on the trailing 2 x 2 block and
// reflector n-3 into A's row n-3 (one block)
__global__ __launch_bounds__(256) void tri_tail_kernel(double *A, int n, double *tv, double *pvb, double *partb,
                                                       double *vbuf, int nblk) {
  __shared__ double s_k;
  const int kp = n - 3, tid = threadIdx.x, lane = tid & 63;
  const double *pvp = pvb + (kp & 1) * (int64_t)n, *ptp = partb + (kp & 1) * (int64_t)nblk;
  const double *vp = vbuf + (kp & 1) * (int64_t)n;
  const double taup = tv[kp];
  if (tid < 64) {
    double acc = 0.0;
    if (taup != 0.0)
      for (int i = lane; i < nblk; i += 64) acc += ptp[i];
    acc = ttk::wave_sum(acc);
    if (lane == 0) s_k = 0.5 * taup * acc;
  }
  __syncthreads();
  const double K = s_k;
  if (tid < 4 && taup != 0.0) {
    const int r = n - 2 + (tid >> 1), j = n - 2 + (tid & 1);
    const int ir = r - kp - 1, jj = j - kp - 1;
    const double vi = vp[ir], wi = pvp[ir] - K * vi, vj = vp[jj];
    A[(int64_t)r * n + j] -= vi * (pvp[jj] - K * vj) + wi * vj;
  }
  for (int j = kp + 1 + tid; j < n; j += 256) A[(int64_t)kp * n + j] = vp[j - kp - 1];
}

// The whole tridiagonalisation of tri_step_hoist_kernel + tri_tail_kernel in ONE workgroup (round 6,
// one launch instead of one per Householder step).  The multi-workgroup form's
// blocks of 4 rows become "virtual blocks": 16 waves take the rows > k round-robin, each row's pending
// update, dot and p entry computed exactly as there (the same expressions, loops and wave reductions),
// and the per-block partial sums of tau p.v are formed in block order from the rows' contributions --
// every stored value and every reduction is the multi-launch path's, so the results are bit-identical
// (tools/dump_kernels.py).  A stays in global memory (L2-resident); the reflector, p and partials live
// in LDS, double-buffered per step as the global vectors were.  NR * 64 >= n - 1 (row elements per lane).
// LDS (doubles): xs n+1 | vb 2n | pvb 2n | crow n.  Four block barriers per step.
template <int NR, int QB>
__global__ __launch_bounds__(1024) void tri_wg_kernel(double *A, int n, double *tv, double *ov, double *dv, int nblk) {
  extern __shared__ double tl[];
  __shared__ double red[16];
  __shared__ double s_k, s_tau_prev;
  double *xs = tl, *vb = xs + n + 1, *pvb = vb + 2 * n, *crow = pvb + 2 * n;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) {
    s_k = 0.0;
    s_tau_prev = 0.0;
  }
  __syncthreads();
  for (int k = 0; k + 2 < n; ++k) {
    const int kp = k - 1, m = n - k - 1;
    const double *pvp = pvb + (kp & 1) * n, *vp = vb + (kp & 1) * n;
    double *pvc = pvb + (k & 1) * n, *vc = vb + (k & 1) * n;
    const double taup = s_tau_prev, K = s_k;
    // ---- row k with step k-1's pending update (tri_step_hoist's expression) and the sigma partials
    // of threads 0..255 (i = 2 + tid + 256 u, the multi-launch block's mapping), from registers
    const double v0 = vp[0], p0 = pvp[0];
    const double wk = taup != 0.0 ? p0 - K * v0 : 0.0, vk = taup != 0.0 ? v0 : 0.0;
    auto rebuilt = [&](int i) {  // xs[i] = A[k, k + i] with the pending update
      const int j = k + i, jj = j - kp - 1;
      double a = A[(int64_t)k * n + j];
      if (taup != 0.0) a -= fma(wk, vp[jj], vk * fma(-K, vp[jj], pvp[jj]));
      return a;
    };
    double part = 0.0;
    if (tid < 256) {
      for (int i = 2 + tid; i <= m; i += 256) {
        const double a = rebuilt(i);
        xs[i] = a;
        part += a * a;
      }
    } else if (tid < 258) {
      xs[tid - 256] = rebuilt(tid - 256);
    }
    if (wid < 4) {
      part = ttk::wave_sum(part);
      if (lane == 0) red[wid] = part;
    }
    __syncthreads();
    double sigma = 0.0;
    for (int i = 0; i < 4; ++i) sigma += red[i];
    const double alpha = xs[1];
    double tau = 0.0, beta = alpha;
    if (sigma > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
      tau = (beta - alpha) / beta;
    }
    const double sc = sigma > 0.0 ? 1.0 / (alpha - beta) : 1.0;
    __syncthreads();  // every thread has read xs[1] and red
    for (int i = 1 + tid; i <= m; i += 1024) {
      const double v = (i == 1) ? 1.0 : xs[i] * sc;
      xs[i] = v;
      vc[i - 1] = v;
    }
    if (tid == 0) {
      tv[k] = tau;
      ov[k] = beta;
      dv[k] = xs[0];
    }
    if (kp >= 0)  // reflector k-1 into A's row k-1 (nobody reads that row again)
      for (int j = k + tid; j < n; j += 1024) A[(int64_t)kp * n + j] = vp[j - k];
    __syncthreads();
    // ---- rows r > k, round-robin over the 16 waves, QB rows' loads in flight per wave; the row-
    // independent operands (reflector k-1, p, reflector k) in registers once per step
    double rv[NR], rp[NR], rx[NR];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      const int j = k + 1 + lane + 64 * u, jj = j - kp - 1;
      rv[u] = j < n ? vp[jj] : 0.0;
      rp[u] = j < n ? pvp[jj] : 0.0;
      rx[u] = j < n ? xs[j - k] : 0.0;
    }
    for (int r0 = k + 1 + wid; r0 < n; r0 += 16 * QB) {
      double ra[QB][NR];
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const int r = r0 + 16 * q;
#pragma unroll
        for (int u = 0; u < NR; ++u) {
          const int j = k + 1 + lane + 64 * u;
          ra[q][u] = (r < n && j < n) ? A[(int64_t)r * n + j] : 0.0;
        }
      }
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const int r = r0 + 16 * q;
        if (r >= n) break;
        const int ir = r - kp - 1;
        const double vi = vp[ir], pi = pvp[ir];
        double *ar = A + (int64_t)r * n;
        const double wi = taup != 0.0 ? pi - K * vi : 0.0, vv = taup != 0.0 ? vi : 0.0;
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < NR; ++u) {
          const int j = k + 1 + lane + 64 * u;
          if (j < n) {
            double a = ra[q][u];
            if (taup != 0.0) {
              a -= fma(wi, rv[u], vv * fma(-K, rv[u], rp[u]));  // tri_step_kernel's contraction
              ar[j] = a;
            }
            acc = fma(a, rx[u], acc);
          }
        }
        acc = ttk::wave_sum(acc);
        if (lane == 0) {
          const double pr = tau * acc;
          pvc[r - k - 1] = pr;
          double contrib = 0.0;
          contrib += pr * xs[r - k];
          crow[r] = contrib;
        }
      }
    }
    __syncthreads();
    // ---- the blocks' partials (rows [4b, 4b+4) above k, in row order, as block_sum adds the waves'
    // values) summed lane-strided in wave 0 for the next step's K, as tri_step_hoist's wave 0 does
    if (wid == 0) {
      double acc = 0.0;
      if (tau != 0.0) {
        for (int b = lane; b < nblk; b += 64) {
          const int rb0 = 4 * b, rb1 = rb0 + 4 < n ? rb0 + 4 : n, rs = rb0 > k + 1 ? rb0 : k + 1;
          double t = 0.0;
          for (int w = 0; w < 4; ++w) {
            const int r = rs + w;
            t += r < rb1 ? crow[r] : 0.0;
          }
          acc += t;
        }
      }
      acc = ttk::wave_sum(acc);
      if (lane == 0) {
        s_k = 0.5 * tau * acc;
        s_tau_prev = tau;
      }
    }
    __syncthreads();
  }
  // ---- tri_tail_kernel: step n-3's pending update of the trailing 2 x 2 block, reflector n-3 into row n-3
  {
    const int kp = n - 3;
    const double *pvp = pvb + (kp & 1) * n, *vp = vb + (kp & 1) * n;
    const double taup = s_tau_prev, K = s_k;
    if (tid < 4 && taup != 0.0) {
      const int r = n - 2 + (tid >> 1), j = n - 2 + (tid & 1);
      const int ir = r - kp - 1, jj = j - kp - 1;
      const double vi = vp[ir], wi = pvp[ir] - K * vi, vj = vp[jj];
      A[(int64_t)r * n + j] -= vi * (pvp[jj] - K * vj) + wi * vj;
    }
    for (int j = kp + 1 + tid; j < n; j += 1024) A[(int64_t)kp * n + j] = vp[j - kp - 1];
  }
}

template <typename K>
void allow_big_lds(K kernel, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// ---------------------------------------------------------------- blocked Householder QR
// Multi-workgroup QR for large matrices (LAPACK dgeqrf + dorgqr structure):
//   panel  : one workgroup factors nb columns (dgeqr2) and forms the nb x nb triangular factor T
//            of the compact-WY form H_j0 ... H_j0+nb-1 = I - Y T Y^T (dlarft, forward/columnwise),
//   apply  : C <- (I - Y op(T) Y^T) C over the chip in two launches: Z = op(T) (Y^T C) (one
//            workgroup per 16 columns, reduction over rows staged through LDS), then C -= Y Z
//            (64 x 16 tiles).  op = T^T applies Q^T (trailing update), op = T applies Q.
// Matrices are column-major with leading dimension ld (column j at base + j*ld).  Y_k is column
// j0+k of the factored matrix with an implicit 1 at row j0+k and zeros above.
constexpr int QB = 32;  // panel width

__device__ __forceinline__ double ycoef(const double *Wf, int ld, int j0, int k, int row) {
  const int d = j0 + k;
  return row < d ? 0.0 : (row == d ? 1.0 : Wf[(int64_t)d * ld + row]);
}

__global__ __launch_bounds__(1024) void qrb_panel_kernel(double *W, int m, int ld, int j0, int nbe,
                                                         double *__restrict__ tau, double *__restrict__ T) {
  __shared__ double red[16];
  __shared__ double ytv[QB];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  for (int e = tid; e < QB * QB; e += nt) T[e] = 0.0;
  for (int jj = 0; jj < nbe; ++jj) {
    const int c = j0 + jj;
    double *x = W + (int64_t)c * ld;
    double part = 0.0;
    for (int i = c + 1 + tid; i < m; i += nt) part += x[i] * x[i];
    const double sigma = ttk::block_sum(part, red);
    const double alpha = x[c];
    double t = 0.0, beta = alpha;
    if (sigma > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
      t = (beta - alpha) / beta;
      const double sc = 1.0 / (alpha - beta);
      for (int i = c + 1 + tid; i < m; i += nt) x[i] *= sc;
    }
    __syncthreads();
    if (tid == 0) {
      x[c] = beta;
      tau[c] = t;
    }
    // apply H_c to the remaining panel columns (one wave per column); v = [1; x[c+1:]]
    for (int c2 = c + 1 + wid; c2 < j0 + nbe; c2 += nw) {
      double *y = W + (int64_t)c2 * ld;
      double acc = 0.0;
      #pragma unroll 8
      for (int i = c + 1 + lane; i < m; i += 64) acc += x[i] * y[i];
      const double w = t * (ttk::wave_sum(acc) + y[c]);
      ttk::axpy_sub_strided(y, x, w, c + 1 + lane, m, 64);
      if (lane == 0) y[c] -= w;
    }
    // T(0:jj, jj) = -t T(0:jj, 0:jj) (Y(:, 0:jj)^T v)
    for (int k = wid; k < jj; k += nw) {
      const double *yk = W + (int64_t)(j0 + k) * ld;
      double acc = 0.0;
      #pragma unroll 8
      for (int i = c + 1 + lane; i < m; i += 64) acc += yk[i] * x[i];
      acc = ttk::wave_sum(acc) + yk[c];
      if (lane == 0) ytv[k] = acc;
    }
    __syncthreads();
    if (tid < jj) {
      double acc = 0.0;
      for (int k = tid; k < jj; ++k) acc += T[tid + k * QB] * ytv[k];
      T[tid + jj * QB] = -t * acc;
    }
    if (tid == 0) T[jj + jj * QB] = t;
    __syncthreads();
  }
}

// Z(0:nbe, 0:ncols) = op(T) Y^T C(:, c0:c0+ncols), rows j0..m-1
__global__ __launch_bounds__(256) void qrb_ytc_kernel(const double *__restrict__ Wf, int m, int ldw, int j0, int nbe,
                                                      const double *__restrict__ C, int ldc, int c0, int ncols,
                                                      const double *__restrict__ T, int transT,
                                                      double *__restrict__ Z) {
  __shared__ double ys[64][QB + 1];
  __shared__ double cs[64][17];
  __shared__ double zs[QB][17];
  __shared__ double ts[QB][QB + 1];
  const int tid = threadIdx.x;
  const int colb = blockIdx.x * 16;
  const int k = tid >> 3, cl = (tid & 7) * 2;  // 32 x 8 threads, 2 columns each
  double acc0 = 0.0, acc1 = 0.0;
  for (int r0 = j0; r0 < m; r0 += 64) {
    for (int e = tid; e < 64 * QB; e += 256) {
      const int rr = e & 63, kk = e >> 6, row = r0 + rr;
      ys[rr][kk] = (row < m && kk < nbe) ? ycoef(Wf, ldw, j0, kk, row) : 0.0;
    }
    for (int e = tid; e < 64 * 16; e += 256) {
      const int rr = e & 63, cc = e >> 6, row = r0 + rr, col = colb + cc;
      cs[rr][cc] = (row < m && col < ncols) ? C[(int64_t)(c0 + col) * ldc + row] : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int rr = 0; rr < 64; ++rr) {
      const double y = ys[rr][k];
      acc0 += y * cs[rr][cl];
      acc1 += y * cs[rr][cl + 1];
    }
    __syncthreads();
  }
  zs[k][cl] = acc0;
  zs[k][cl + 1] = acc1;
  for (int e = tid; e < QB * QB; e += 256) {
    const int i = e & (QB - 1), j = e / QB;
    ts[i][j] = transT ? T[j + i * QB] : T[i + j * QB];  // op(T)(i, j)
  }
  __syncthreads();
  double o0 = 0.0, o1 = 0.0;
  for (int j = 0; j < nbe; ++j) {
    const double tij = ts[k][j];
    o0 += tij * zs[j][cl];
    o1 += tij * zs[j][cl + 1];
  }
  if (k < nbe) {
    if (colb + cl < ncols) Z[(int64_t)(colb + cl) * QB + k] = o0;
    if (colb + cl + 1 < ncols) Z[(int64_t)(colb + cl + 1) * QB + k] = o1;
  }
}

// C(j0:m, c0:c0+ncols) -= Y Z
__global__ __launch_bounds__(256) void qrb_update_kernel(const double *__restrict__ Wf, int m, int ldw, int j0,
                                                         int nbe, double *__restrict__ C, int ldc, int c0, int ncols,
                                                         const double *__restrict__ Z) {
  __shared__ double ys[64][QB + 1];
  __shared__ double zs[QB][17];
  const int tid = threadIdx.x;
  const int r0 = j0 + blockIdx.x * 64, colb = blockIdx.y * 16;
  for (int e = tid; e < 64 * QB; e += 256) {
    const int rr = e & 63, kk = e >> 6, row = r0 + rr;
    ys[rr][kk] = (row < m && kk < nbe) ? ycoef(Wf, ldw, j0, kk, row) : 0.0;
  }
  for (int e = tid; e < QB * 16; e += 256) {
    const int kk = e & (QB - 1), cc = e / QB, col = colb + cc;
    zs[kk][cc] = (kk < nbe && col < ncols) ? Z[(int64_t)col * QB + kk] : 0.0;
  }
  __syncthreads();
  const int cc = tid & 15, rb = (tid >> 4) * 4;
  const int col = colb + cc;
  if (col >= ncols) return;
  double *cp = C + (int64_t)(c0 + col) * ldc;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = rb + i, row = r0 + rr;
    if (row >= m) break;
    double acc = 0.0;
    for (int kk = 0; kk < nbe; ++kk) acc += ys[rr][kk] * zs[kk][cc];
    cp[row] -= acc;
  }
}

// dst(rows x cols, row-major ldd) = src viewed column-major (ld lds) [transposed read] or copy
__global__ void cm_to_rm_kernel(const double *__restrict__ src, int lds, double *__restrict__ dst, int rows,
                                int cols) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)rows * cols;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / cols), j = (int)(e - (int64_t)i * cols);
    dst[e] = src[(int64_t)j * lds + i];
  }
}

// A (m x n row-major) -> W (column-major, ld = m)
__global__ void rm_to_cm_kernel(const double *__restrict__ A, int m, int n, double *__restrict__ W) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)m * n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(e / m), i = (int)(e - (int64_t)j * m);
    W[e] = A[(int64_t)i * n + j];
  }
}

// M (column-major q x p, ld q) = [Vt^T ; 0] where Vt is p x p row-major (column j of M = row j of Vt)
// or [I; 0] when Vt == nullptr
__global__ void qpad_kernel(const double *__restrict__ Vt, int p, int q, int k, double *__restrict__ M) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)q * k;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(e / q), i = (int)(e - (int64_t)j * q);
    M[e] = Vt ? (i < p ? Vt[(int64_t)j * p + i] : 0.0) : (i == j ? 1.0 : 0.0);
  }
}

// X (p x p column-major) = R^T where R = upper triangle of W's first p rows; V = I
__global__ void rt_build_kernel(const double *__restrict__ W, int ld, int p, double *__restrict__ X,
                                double *__restrict__ V) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)p * p;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(e / p), k = (int)(e - (int64_t)j * p);  // X(k, j) = R(j, k)
    X[e] = (k >= j) ? W[(int64_t)k * ld + j] : 0.0;
    V[e] = (j == k) ? 1.0 : 0.0;
  }
}

// R (k x n row-major) = upper triangle of W (col-major, ld m)
__global__ void r_extract_kernel(const double *__restrict__ W, int ld, int k, int n, double *__restrict__ R) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)k * n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / n), j = (int)(e - (int64_t)i * n);
    R[e] = (j >= i) ? W[(int64_t)j * ld + i] : 0.0;
  }
}

// ------------------------------------------------------ QR with column pivoting (dgeqp3)
// Per column c: one workgroup picks the pivot (first max of the downdated norms, idamax), swaps
// it in and forms the Householder reflector; then one launch applies the reflector to every
// trailing column (one wave per column) and downdates its norm with LAPACK's dlaqp2 rule
// (recompute when the downdate loses more than sqrt(eps)).  Column pivoting makes R's rows
// graded, which is what lets the one-sided Jacobi on R^T converge in ~10 sweeps on the path's
// unfoldings (41+ without it; Drmac-Veselic preconditioning).  Optional deflation: stop when the
// remaining Frobenius norm is <= defl (the caller's truncation tolerance x 1e-3).
// ctl[0] = effective rank, ctl[1] = stopped flag.
__global__ __launch_bounds__(256) void qrcp_init_kernel(const double *__restrict__ W, int m, int n,
                                                        double *__restrict__ vn1, double *__restrict__ vn2,
                                                        int *__restrict__ perm, int *__restrict__ ctl, int k) {
  const int j = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctl[0] = k;
    ctl[1] = 0;
  }
  if (j >= n) return;
  const double *w = W + (int64_t)j * m;
  double acc = 0.0;
  #pragma unroll 8
  for (int i = lane; i < m; i += 64) acc += w[i] * w[i];
  acc = sqrt(ttk::wave_sum(acc));
  if (lane == 0) {
    vn1[j] = acc;
    vn2[j] = acc;
    perm[j] = j;
  }
}

__global__ __launch_bounds__(1024) void qrcp_pivot_kernel(double *W, int m, int n, int c, double *vn1, double *vn2,
                                                          int *perm, double *__restrict__ tau, int *ctl, double defl2) {
  __shared__ double smax[16], ssum[16], red[16];
  __shared__ int sidx[16];
  __shared__ int s_piv, s_stop;
  if (ctl[1]) return;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  double bm = -1.0, sum = 0.0;
  int bi = n;
  for (int j = c + tid; j < n; j += nt) {
    const double v = vn1[j];
    sum += v * v;
    if (v > bm) {  // strided scan: first max within this thread's subsequence
      bm = v;
      bi = j;
    }
  }
  // wave reduction of (max, first index) and the sum
  ttk::wave_argmax(bm, bi);
  sum = ttk::wave_sum(sum);
  if (lane == 0) {
    smax[wid] = bm;
    sidx[wid] = bi;
    ssum[wid] = sum;
  }
  __syncthreads();
  if (tid == 0) {
    double m0 = -1.0, s0 = 0.0;
    int i0 = n;
    for (int w = 0; w < nw; ++w) {
      s0 += ssum[w];
      if (smax[w] > m0 || (smax[w] == m0 && sidx[w] < i0)) {
        m0 = smax[w];
        i0 = sidx[w];
      }
    }
    s_stop = (defl2 > 0.0 && s0 <= defl2) || s0 == 0.0;
    s_piv = i0;
    if (s_stop) {
      ctl[0] = c;
      ctl[1] = 1;
    }
  }
  __syncthreads();
  if (s_stop) return;
  const int piv = s_piv;
  if (piv != c) {
    double *a = W + (int64_t)c * m, *b = W + (int64_t)piv * m;
    for (int i = tid; i < m; i += nt) {
      const double t = a[i];
      a[i] = b[i];
      b[i] = t;
    }
    if (tid == 0) {
      double t = vn1[c];
      vn1[c] = vn1[piv];
      vn1[piv] = t;
      t = vn2[c];
      vn2[c] = vn2[piv];
      vn2[piv] = t;
      const int pi = perm[c];
      perm[c] = perm[piv];
      perm[piv] = pi;
    }
    __syncthreads();
  }
  double *x = W + (int64_t)c * m;
  double part = 0.0;
  for (int i = c + 1 + tid; i < m; i += nt) part += x[i] * x[i];
  const double sigma = ttk::block_sum(part, red);
  const double alpha = x[c];
  double t = 0.0, beta = alpha;
  if (sigma > 0.0) {
    beta = -copysign(sqrt(alpha * alpha + sigma), alpha);
    t = (beta - alpha) / beta;
    const double sc = 1.0 / (alpha - beta);
    for (int i = c + 1 + tid; i < m; i += nt) x[i] *= sc;
  }
  __syncthreads();  // every thread has read alpha = x[c] before it is overwritten
  if (tid == 0) {
    x[c] = beta;
    tau[c] = t;
  }
  (void)wid;
}

__global__ __launch_bounds__(256) void qrcp_update_kernel(double *__restrict__ W, int m, int n, int c,
                                                          double *__restrict__ vn1, double *__restrict__ vn2,
                                                          const double *__restrict__ tau, const int *__restrict__ ctl) {
  if (ctl[1]) return;
  const int j = c + 1 + (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= n) return;
  const double t = tau[c];
  const double *v = W + (int64_t)c * m;
  double *y = W + (int64_t)j * m;
  double yc = y[c];
  if (t != 0.0) {
    double acc = 0.0;
    #pragma unroll 8
    for (int i = c + 1 + lane; i < m; i += 64) acc += v[i] * y[i];
    const double w = t * (ttk::wave_sum(acc) + yc);
    ttk::axpy_sub_strided(y, v, w, c + 1 + lane, m, 64);
    yc -= w;
    if (lane == 0) y[c] = yc;
  }
  const double a = vn1[j];
  if (a != 0.0) {  // dlaqp2 norm downdate
    double temp = fabs(yc) / a;
    temp = fmax(1.0 - temp * temp, 0.0);
    const double r = a / vn2[j];
    if (temp * r * r <= 1.4901161193847656e-08) {
      double acc = 0.0;
      #pragma unroll 8
      for (int i = c + 1 + lane; i < m; i += 64) acc += y[i] * y[i];
      acc = sqrt(ttk::wave_sum(acc));
      if (lane == 0) {
        vn1[j] = acc;
        vn2[j] = acc;
      }
    } else if (lane == 0) {
      vn1[j] = a * sqrt(temp);
    }
  }
}

// T factors (dlarft, forward/columnwise) of every QB-panel of reflectors 0..kk-1 stored in W
__global__ __launch_bounds__(256) void tfactor_kernel(const double *__restrict__ W, int m, int kk,
                                                      const double *__restrict__ tau, double *__restrict__ Tall) {
  __shared__ double ytv[QB];
  const int pi = blockIdx.x, j0 = pi * QB;
  const int nbe = (kk - j0) < QB ? (kk - j0) : QB;
  double *T = Tall + (int64_t)pi * QB * QB;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  for (int e = tid; e < QB * QB; e += nt) T[e] = 0.0;
  __syncthreads();
  for (int jj = 0; jj < nbe; ++jj) {
    const int c = j0 + jj;
    const double t = tau[c];
    const double *x = W + (int64_t)c * m;
    for (int k = wid; k < jj; k += nw) {
      const double *yk = W + (int64_t)(j0 + k) * m;
      double acc = 0.0;
      #pragma unroll 8
      for (int i = c + 1 + lane; i < m; i += 64) acc += yk[i] * x[i];
      acc = ttk::wave_sum(acc) + yk[c];
      if (lane == 0) ytv[k] = acc;
    }
    __syncthreads();
    if (tid < jj) {
      double acc = 0.0;
      for (int k = tid; k < jj; ++k) acc += T[tid + k * QB] * ytv[k];
      T[tid + jj * QB] = -t * acc;
    }
    if (tid == 0) T[jj + jj * QB] = t;
    __syncthreads();
  }
}

// X (col-major, column length p, kk columns) = R1^T, R1 = first kk rows of the upper triangle of
// W (col-major, ld m); V = I (kk x kk)
__global__ void rt_build2_kernel(const double *__restrict__ W, int ld, int p, int kk, double *__restrict__ X,
                                 double *__restrict__ V) {
  const int64_t tx = (int64_t)kk * p, tv = (int64_t)kk * kk;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tx + tv; e += (int64_t)gridDim.x * blockDim.x) {
    if (e < tx) {
      const int i = (int)(e / p), j = (int)(e - (int64_t)i * p);  // X(j, i) = R(i, j)
      X[e] = (j >= i) ? W[(int64_t)j * ld + i] : 0.0;
    } else {
      const int64_t f = e - tx;
      V[f] = ((f / kk) == (f % kk)) ? 1.0 : 0.0;
    }
  }
}

// final assembly: Lw = M (col-major q x kk), Rw = P Ux (Ux row-major p x kk, perm[i] = original
// column of pivoted column i); tall: U = Lw, Vt = Rw^T; wide: U = Rw, Vt = Lw^T; rank >= kk zero
__global__ void svd_big_out_kernel(const double *__restrict__ M, const double *__restrict__ Ux,
                                   const int *__restrict__ perm, int q, int p, int kk, int tall,
                                   double *__restrict__ U, double *__restrict__ Vt, double *__restrict__ S) {
  const int64_t nl = (int64_t)q * p, nr = (int64_t)p * p;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nl + nr + p;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e < nl) {  // left factor of W: element (i, r), i < q, r < p
      const int i = (int)(e / p), r = (int)(e - (int64_t)i * p);
      const double v = r < kk ? M[(int64_t)r * q + i] : 0.0;
      if (tall)
        U[(int64_t)i * p + r] = v;        // U (q x p)
      else
        Vt[(int64_t)r * q + i] = v;       // Vt (p x q)
    } else if (e < nl + nr) {  // right factor of W: element (perm[i], r)
      const int64_t f = e - nl;
      const int i = (int)(f / p), r = (int)(f - (int64_t)i * p);
      const double v = r < kk ? Ux[(int64_t)i * kk + r] : 0.0;
      const int oi = perm[i];
      if (tall)
        Vt[(int64_t)r * p + oi] = v;      // Vt (p x p)
      else
        U[(int64_t)oi * p + r] = v;       // U (p x p)
    } else {
      const int r = (int)(e - nl - nr);
      if (r >= kk) S[r] = 0.0;
    }
  }
}

inline int grid_for(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

// factor W (m x n col-major, ld m) in place: R in the upper triangle, reflectors below, tau (k),
// T factors (QB x QB each) per panel
int qrb_factor(hipStream_t st, double *W, int m, int n, double *tau, double *Tall, double *Z) {
  const int k = m < n ? m : n;
  for (int j0 = 0; j0 < k; j0 += QB) {
    const int nbe = (k - j0) < QB ? (k - j0) : QB;
    double *T = Tall + (int64_t)(j0 / QB) * QB * QB;
    hipLaunchKernelGGL(qrb_panel_kernel, dim3(1), dim3(1024), 0, st, W, m, m, j0, nbe, tau, T);
    TTK_LAUNCH_CHECK();
    const int c0 = j0 + nbe, nc = n - c0;
    if (nc > 0) {
      hipLaunchKernelGGL(qrb_ytc_kernel, dim3((nc + 15) / 16), dim3(256), 0, st, W, m, m, j0, nbe, W, m, c0, nc, T, 1,
                         Z);
      hipLaunchKernelGGL(qrb_update_kernel, dim3((m - j0 + 63) / 64, (nc + 15) / 16), dim3(256), 0, st, W, m, m, j0,
                         nbe, W, m, c0, nc, Z);
      TTK_LAUNCH_CHECK();
    }
  }
  return TTK_OK;
}

// M (m x nc col-major, ld m) <- Q M with Q = H_0 ... H_{k-1} from qrb_factor
int qrb_apply_q(hipStream_t st, const double *W, int m, int k, const double *Tall, double *M, int nc, double *Z) {
  const int npan = (k + QB - 1) / QB;
  for (int pi = npan - 1; pi >= 0; --pi) {
    const int j0 = pi * QB, nbe = (k - j0) < QB ? (k - j0) : QB;
    const double *T = Tall + (int64_t)pi * QB * QB;
    hipLaunchKernelGGL(qrb_ytc_kernel, dim3((nc + 15) / 16), dim3(256), 0, st, W, m, m, j0, nbe, M, m, 0, nc, T, 0, Z);
    hipLaunchKernelGGL(qrb_update_kernel, dim3((m - j0 + 63) / 64, (nc + 15) / 16), dim3(256), 0, st, W, m, m, j0, nbe,
                       M, m, 0, nc, Z);
    TTK_LAUNCH_CHECK();
  }
  return TTK_OK;
}

int ensure_status() {  // the current context's device status words
  ttk::Ctx &c = ttk::ctx();
  if (!c.status) {
    if (hipMalloc(reinterpret_cast<void **>(&c.status), 16 * sizeof(int)) != hipSuccess) return TTK_ERR_HIP;
    if (hipMalloc(reinterpret_cast<void **>(&c.rcond), 16 * sizeof(double)) != hipSuccess) return TTK_ERR_HIP;
  }
  return TTK_OK;
}

}  // namespace

extern "C" {

static int g_svd_big_p = 64;
static int g_svd_timing = 0;  // phase timers of the one-workgroup SVD into the debug counters

// diagnostics: shape histogram of the dense factorisations (ttk_linalg_hist).  While on, each
// recorded call is bracketed by two stream synchronisations and its wall time (launch overhead
// included) added to its (kind, a, b, path) entry -- a sizing tool, never on in a timed run.
namespace {
bool g_lhist_on = false;
std::mutex g_lhist_mu;
std::map<std::array<int, 4>, std::pair<long long, double>> g_lhist;
const char *const LHIST_KIND[] = {"svd", "qr", "syev_extreme", "lu", "cholesky"};
struct LinalgScope {
  hipStream_t st;
  std::array<int, 4> key;
  std::chrono::steady_clock::time_point t0;
  LinalgScope(hipStream_t s, int kind, int a, int b, int path) : st(s), key{kind, a, b, path} {
    if (!g_lhist_on) return;
    (void)hipStreamSynchronize(st);
    t0 = std::chrono::steady_clock::now();
  }
  ~LinalgScope() {
    if (!g_lhist_on) return;
    (void)hipStreamSynchronize(st);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    std::lock_guard<std::mutex> lk(g_lhist_mu);
    auto &e = g_lhist[key];
    e.first += 1;
    e.second += us;
  }
};
}  // namespace

int ttk_linalg_hist(int on, const char *dump_path) {
  std::lock_guard<std::mutex> lk(g_lhist_mu);
  if (dump_path) {
    FILE *f = std::fopen(dump_path, "w");
    if (!f) return TTK_ERR_ARG;
    std::fprintf(f, "kind a b path calls total_us\n");
    for (const auto &kv : g_lhist)
      std::fprintf(f, "%s %d %d %d %lld %.1f\n", LHIST_KIND[kv.first[0]], kv.first[1], kv.first[2], kv.first[3],
                   kv.second.first, kv.second.second);
    std::fclose(f);
  }
  if (on < 0) g_lhist.clear();
  g_lhist_on = on > 0;
  return TTK_OK;
}

int ttk_svd_set_timing(int on) {
  const int old = g_svd_timing;
  g_svd_timing = on;
  return old;
}  // smallest p that takes the multi-workgroup path (when W does not fit LDS)

static int64_t svd_big_work(int m, int n) {
  const int64_t p = m < n ? m : n, q = m < n ? n : m, npan = (p + QB - 1) / QB;
  return 2 * q * p + 4 * p * p + 6 * p + npan * QB * QB + QB * p + 64;
}

// Large SVD: W P = Q R by column-pivoted Householder QR (optionally deflated at `defl`), one-sided
// Jacobi on X = R1^T (p x k_eff; QRCP makes it converge in ~10 sweeps), then the left vectors
// Q [V_X; 0] and the right vectors P U_X.  W = A (tall) or A^T (wide).
static int svd_big(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt, double *work,
                   double defl) {
  int rc = ensure_status();
  if (rc != TTK_OK) return rc;
  const bool tall = m >= n;
  const int p = tall ? n : m, q = tall ? m : n;
  const int npan = (p + QB - 1) / QB;
  double *W = work;                                  // q x p col-major
  double *M = W + (int64_t)q * p;                    // q x p col-major
  double *X = M + (int64_t)q * p;                    // p x p col-major (k_eff columns used)
  double *V = X + (int64_t)p * p;                    // k_eff x k_eff
  double *Ux = V + (int64_t)p * p;                   // p x k_eff row-major
  double *VtX = Ux + (int64_t)p * p;                 // k_eff x k_eff row-major
  double *tau = VtX + (int64_t)p * p;                // p
  double *vn1 = tau + p, *vn2 = vn1 + p;             // p, p
  double *sig = vn2 + p;                             // p
  int *rank = reinterpret_cast<int *>(sig + p);      // p ints
  int *perm = reinterpret_cast<int *>(sig + 2 * p);  // p ints
  double *Tall = sig + 3 * p;                        // npan * QB * QB
  double *Z = Tall + (int64_t)npan * QB * QB;        // QB * p
  int *ctl = ttk::ctx().status + 10;                          // [0] k_eff, [1] stopped
  int *flag = ttk::ctx().status + 8;
  hipStream_t st = TTK_STREAM(stream);
  if (tall)
    hipLaunchKernelGGL(rm_to_cm_kernel, dim3(grid_for((int64_t)q * p)), dim3(256), 0, st, A, m, n, W);
  else  // W = A^T: column j of W = row j of A -> a plain copy
    TTK_HIP(hipMemcpyAsync(W, A, sizeof(double) * (size_t)q * p, hipMemcpyDeviceToDevice, st));
  TTK_LAUNCH_CHECK();
  const double defl2 = defl > 0.0 ? defl * defl : 0.0;
  hipLaunchKernelGGL(qrcp_init_kernel, dim3((p * 64 + 255) / 256), dim3(256), 0, st, W, q, p, vn1, vn2, perm, ctl, p);
  TTK_LAUNCH_CHECK();
  for (int c = 0; c < p; ++c) {
    hipLaunchKernelGGL(qrcp_pivot_kernel, dim3(1), dim3(1024), 0, st, W, q, p, c, vn1, vn2, perm, tau, ctl, defl2);
    if (c + 1 < p)
      hipLaunchKernelGGL(qrcp_update_kernel, dim3(((p - c - 1) * 64 + 255) / 256), dim3(256), 0, st, W, q, p, c, vn1,
                         vn2, tau, ctl);
    TTK_LAUNCH_CHECK();
    if ((c & 63) == 63 && c + 1 < p) {  // early-exit check for deflated solves
      int h = 0;
      TTK_HIP(hipMemcpyAsync(&h, ctl + 1, sizeof(int), hipMemcpyDeviceToHost, st));
      ttk::note_sync();
      TTK_HIP(hipStreamSynchronize(st));
      if (h) break;
    }
  }
  int hk[2] = {p, 0};
  TTK_HIP(hipMemcpyAsync(hk, ctl, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
  ttk::note_sync();
  TTK_HIP(hipStreamSynchronize(st));
  const int kk = hk[0] < 1 ? 1 : hk[0];  // keep one direction so the epilogue is well defined
  const int nkp = (kk + QB - 1) / QB;
  hipLaunchKernelGGL(tfactor_kernel, dim3(nkp), dim3(256), 0, st, W, q, kk, tau, Tall);
  hipLaunchKernelGGL(rt_build2_kernel, dim3(grid_for((int64_t)kk * (p + kk))), dim3(256), 0, st, W, q, p, kk, X, V);
  TTK_LAUNCH_CHECK();
  const double tol = EPS * (p > 16 ? (double)p : 16.0);
  const int P = (kk % 2) ? kk + 1 : kk;
  const int grid = (P / 2 * 64 + 255) / 256;
  ttk::Ctx &cx = ttk::ctx();
  const bool one = cx.knob[TTK_KNOB_SVD_SWEEP_ONE] != 0 && kk > 1;
  if (one) {  // per-column round counters (zeroed per SVD) and the context's hand-off words
    if (cx.colr_n < P) {
      if (cx.colr) (void)hipFree(cx.colr);
      cx.colr = nullptr;
      cx.colr_n = 0;
      TTK_HIP(hipMalloc(reinterpret_cast<void **>(&cx.colr), sizeof(unsigned) * (size_t)P));
      cx.colr_n = P;
    }
    TTK_HIP(hipMemsetAsync(cx.colr, 0, sizeof(unsigned) * (size_t)P, st));
    rc = ttk::dep_counter(stream);
    if (rc != TTK_OK) return rc;
  }
  for (int sweep = 0; sweep < 60 && kk > 1; ++sweep) {
    TTK_HIP(hipMemsetAsync(flag, 0, sizeof(int), st));
    if (one) {
      hipLaunchKernelGGL(svd_big_sweep_kernel, dim3(grid), dim3(256), 0, st, X, V, kk, p, tol, flag, cx.colr,
                         (unsigned)sweep * (unsigned)(P - 1), cx.dep, cx.tick_total);
      cx.tick_total += (unsigned)grid;
    } else {
      for (int r = 0; r < P - 1; ++r)
        hipLaunchKernelGGL(svd_big_round_kernel, dim3(grid), dim3(256), 0, st, X, V, kk, p, r, tol, flag);
    }
    TTK_LAUNCH_CHECK();
    int h = 0;
    TTK_HIP(hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, st));
    ttk::note_sync();
    TTK_HIP(hipStreamSynchronize(st));
    if (!h) break;
  }
  // X (p x kk) = U_X S V_X^T: Ux (p x kk row-major), S[0:kk], VtX (kk x kk row-major)
  hipLaunchKernelGGL(svd_big_finish_kernel, dim3(1), dim3(1024), 0, st, X, V, sig, rank, p, kk, Ux, S, VtX);
  TTK_LAUNCH_CHECK();
  // M = Q [V_X; 0]  (q x kk)
  hipLaunchKernelGGL(qpad_kernel, dim3(grid_for((int64_t)q * kk)), dim3(256), 0, st, VtX, kk, q, kk, M);
  TTK_LAUNCH_CHECK();
  rc = qrb_apply_q(st, W, q, kk, Tall, M, kk, Z);
  if (rc != TTK_OK) return rc;
  hipLaunchKernelGGL(svd_big_out_kernel, dim3(grid_for((int64_t)q * p + (int64_t)p * p + p)), dim3(256), 0, st, M, Ux,
                     perm, q, p, kk, tall ? 1 : 0, U, Vt, S);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

static int64_t qr_big_work(int m, int n) {
  const int64_t k = m < n ? m : n, npan = (k + QB - 1) / QB, mx = m > n ? m : n;
  return (int64_t)m * n + (int64_t)m * k + k + npan * QB * QB + QB * mx + 64;
}

static int qr_big(void *stream, const double *A, int m, int n, double *Q, double *R, double *work) {
  const int k = m < n ? m : n, npan = (k + QB - 1) / QB;
  double *W = work, *M = W + (int64_t)m * n, *tau = M + (int64_t)m * k, *Tall = tau + k;
  double *Z = Tall + (int64_t)npan * QB * QB;
  hipStream_t st = TTK_STREAM(stream);
  hipLaunchKernelGGL(rm_to_cm_kernel, dim3(grid_for((int64_t)m * n)), dim3(256), 0, st, A, m, n, W);
  TTK_LAUNCH_CHECK();
  int rc = qrb_factor(st, W, m, n, tau, Tall, Z);
  if (rc != TTK_OK) return rc;
  hipLaunchKernelGGL(qpad_kernel, dim3(grid_for((int64_t)m * k)), dim3(256), 0, st, nullptr, k, m, k, M);
  TTK_LAUNCH_CHECK();
  rc = qrb_apply_q(st, W, m, k, Tall, M, k, Z);
  if (rc != TTK_OK) return rc;
  hipLaunchKernelGGL(cm_to_rm_kernel, dim3(grid_for((int64_t)m * k)), dim3(256), 0, st, M, m, Q, m, k);
  hipLaunchKernelGGL(r_extract_kernel, dim3(grid_for((int64_t)k * n)), dim3(256), 0, st, W, m, k, n, R);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_svd_set_big_threshold(int p) {
  const int old = g_svd_big_p;
  if (p > 0) g_svd_big_p = p;
  return old;
}

int64_t ttk_svd_work(int m, int n) {
  const int64_t p = m < n ? m : n, q = m < n ? n : m;
  const int64_t small = 2 * (q | 1) * p + 16, big = svd_big_work(m, n);
  return small > big ? small : big;
}

int ttk_svd(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt, double *work) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  return ttk_svd_tol(stream, A, m, n, U, S, Vt, work, 0.0);
}

static int svd_tol_impl(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt,
                        double *work, double defl, double *host_s);

int ttk_svd_tol(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt, double *work,
                double defl) {
  return svd_tol_impl(stream, A, m, n, U, S, Vt, work, defl, nullptr);
}


int ttk_svd_tol_read(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt,
                     double *work, double defl, double *s_host) {
  if (!s_host) {
    ttk::set_error("ttk_svd_tol_read: null host buffer");
    return TTK_ERR_ARG;
  }
  const int64_t k = m < n ? m : n;
  double *hdev = nullptr, *h = k > 0 && k <= 65536 ? ttk::mapped_stage((size_t)k, &hdev) : nullptr;
  int rc = h ? svd_tol_impl(stream, A, m, n, U, S, Vt, work, defl, hdev) : TTK_ERR_ARG;
  if (rc == TTK_OK) {
    ttk::note_sync();
    TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
    std::memcpy(s_host, h, (size_t)k * sizeof(double));
    return TTK_OK;
  }
  if (rc != TTK_ERR_ARG || m <= 0 || n <= 0) return rc;
  rc = svd_tol_impl(stream, A, m, n, U, S, Vt, work, defl, nullptr);  // the multi-workgroup path
  return rc ? rc : ttk_read_sync(stream, S, s_host, k);
}

static int svd_tol_impl(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt,
                        double *work, double defl, double *host_s) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (m <= 0 || n <= 0) {
    ttk::set_error("ttk_svd: empty matrix %dx%d", m, n);
    return TTK_ERR_ARG;
  }
  const int p = m < n ? m : n, q = m < n ? n : m;
  const bool forced_big = g_svd_big_p <= 2;
  if (host_s && (p > WG_P || forced_big)) return TTK_ERR_ARG;  // the caller reads S itself
  LinalgScope scope_(TTK_STREAM(stream), 0, m, n, p > WG_P || forced_big ? 0 : -1);
  if (p > WG_P || forced_big) return svd_big(stream, A, m, n, U, S, Vt, work, defl);
  // small near-square problems converge fast without QR preconditioning; otherwise QRCP first
  const int use_qr = !(p <= 16 && q <= 2 * p);
  const int L = use_qr ? p : q;
  const int64_t fixed = (int64_t)(L | 1) * p + (int64_t)(p | 1) * p + 5 * (int64_t)p + 2;  // X, V, vectors
  const int64_t wm = use_qr ? 2 * (int64_t)(q | 1) * p : 0;                    // W and M (odd stride)
  // W and M in LDS (2), W alone (1: M in the global working buffer), neither (0); mode 1 only for the
  // instantiated lanes-per-pair counts (4, 8, 16: the p that overflow LDS with both)
  int wmode = fixed + wm <= LDS_DOUBLES ? 2 : (use_qr && fixed + wm / 2 <= LDS_DOUBLES ? 1 : 0);
  const int w_in_lds = wmode == 2;

  const int pairs = (p + 1) / 2;
  int g = 1;
  while (g < 64 && g * VPL < L) g *= 2;  // <= VPL elements of a column per lane
  int nt = pairs * g;
  if (use_qr && q * p > 2048) nt = 1024;  // column-parallel QR phases want a full block
  nt = nt < 64 ? 64 : (nt > 1024 ? 1024 : (nt + 63) / 64 * 64);
  if (wmode == 1 && !(g == 4 || g == 8 || g == 16)) wmode = 0;
  const size_t shm = (size_t)(fixed + (wmode == 2 ? wm : wmode == 1 ? wm / 2 : 0)) * sizeof(double);
  // path: svd_wg_kernel<g>, sign = QRCP, x100 = W global, x10 = W in LDS and M global
  scope_.key[3] = g * (use_qr ? 1 : -1) * (wmode == 2 ? 1 : wmode == 1 ? 10 : 100);
  (void)defl;  // no deflation on this path (every direction keeps an orthonormal vector)
#define TTK_SVD_WG_MODE(GG, MM)                                                                             \
  {                                                                                                         \
    allow_big_lds(svd_wg_kernel<GG, MM>, shm);                                                              \
    hipLaunchKernelGGL((svd_wg_kernel<GG, MM>), dim3(1), dim3(nt), shm, TTK_STREAM(stream), A, m, n, U, S, Vt, \
                       work, w_in_lds, use_qr, g_svd_timing, host_s);                                          \
  }
#define TTK_SVD_WG(GG)                                                                                      \
  case GG:                                                                                                  \
    if (wmode == 2) TTK_SVD_WG_MODE(GG, 2) else TTK_SVD_WG_MODE(GG, 0)                                       \
    break;
#define TTK_SVD_WG3(GG)                                                                                     \
  case GG:                                                                                                  \
    if (wmode == 2) TTK_SVD_WG_MODE(GG, 2) else if (wmode == 1) TTK_SVD_WG_MODE(GG, 1) else TTK_SVD_WG_MODE(GG, 0) \
    break;
  switch (g) {
    TTK_SVD_WG(1)
    TTK_SVD_WG(2)
    TTK_SVD_WG3(4)
    TTK_SVD_WG3(8)
    TTK_SVD_WG3(16)
    TTK_SVD_WG(32)
    default:
      TTK_SVD_WG(64)
  }
#undef TTK_SVD_WG
#undef TTK_SVD_WG3
#undef TTK_SVD_WG_MODE
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

static const int g_qr_narrow = getenv("TTK_QR_NARROW") ? atoi(getenv("TTK_QR_NARROW")) : 1;
static int g_qr_big_k = 48;  // smallest min(m,n) that takes the blocked path (when it does not fit LDS)

int ttk_qr_set_big_threshold(int k) {
  const int old = g_qr_big_k;
  if (k > 0) g_qr_big_k = k;
  return old;
}

int64_t ttk_qr_work(int m, int n) {
  const int64_t k = m < n ? m : n;
  const int64_t small = (int64_t)m * n + k + (int64_t)m * k + 16, big = qr_big_work(m, n);
  return small > big ? small : big;
}

static int qr_impl(void *stream, const double *A, int m, int n, double *Q, double *R, double *work,
                   int colmajor);

int ttk_qr(void *stream, const double *A, int m, int n, double *Q, double *R, double *work) {
  return qr_impl(stream, A, m, n, Q, R, work, 0);
}

}  // extern "C"
namespace ttk {
// ttk_qr on A^T (row-major n x m, i.e. A column-major) returning Q^T (k x m row-major) and R as
// ttk_qr does; TTK_ERR_ARG without launching anything when the shape takes the blocked path
int qr_colmajor(void *stream, const double *At, int m, int n, double *Qt, double *R, double *work) {
  return qr_impl(stream, At, m, n, Qt, R, work, 1);
}
}  // namespace ttk
extern "C" {

static int qr_impl(void *stream, const double *A, int m, int n, double *Q, double *R, double *work,
                   int colmajor) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (m <= 0 || n <= 0) {
    ttk::set_error("ttk_qr: empty matrix %dx%d", m, n);
    return TTK_ERR_ARG;
  }
  const int64_t k = m < n ? m : n;
  const int64_t need = (int64_t)m * n + k + (int64_t)m * k + 16;
  const int use_lds = need <= LDS_DOUBLES;
  if (colmajor && k >= g_qr_big_k && (!use_lds || g_qr_big_k <= 2)) return TTK_ERR_ARG;  // caller transposes
  LinalgScope scope_(TTK_STREAM(stream), 1, m, n, k >= g_qr_big_k && (!use_lds || g_qr_big_k <= 2) ? 0 : use_lds ? 1 : 2);
  if (k >= g_qr_big_k && (!use_lds || g_qr_big_k <= 2)) return qr_big(stream, A, m, n, Q, R, work);
  const size_t shm = use_lds ? need * sizeof(double) : 0;
  // m <= 65: every thread's norm chain holds at most one element whatever the block size, and the
  // per-column work is one wave's either way, so one wave per trailing column (<= 16) computes the
  // same bits as the full 1024-thread block with fewer waves to synchronise (TTK_QR_NARROW=0: 1024)
  const int nt = (g_qr_narrow && m <= 65) ? 64 * (n < 16 ? (n < 1 ? 1 : n) : 16) : 1024;
  if (use_lds) {
    allow_big_lds(qr_kernel<true>, shm);
    hipLaunchKernelGGL(qr_kernel<true>, dim3(1), dim3(nt), shm, TTK_STREAM(stream), A, m, n, Q, R, work, use_lds, colmajor);
  } else {
    allow_big_lds(qr_kernel<false>, shm);
    hipLaunchKernelGGL(qr_kernel<false>, dim3(1), dim3(nt), shm, TTK_STREAM(stream), A, m, n, Q, R, work, use_lds, colmajor);
  }
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

static int g_dense_block_min = 96;  // n at or above which Cholesky / TRSM take the blocked kernels
static int g_lu_block_min = getenv("TTK_LU_BLOCK_MIN") ? atoi(getenv("TTK_LU_BLOCK_MIN")) : 32;  // LU / getrs

int ttk_dense_set_block_min(int n) {
  const int old = g_dense_block_min;
  g_dense_block_min = n;
  return old;
}

int ttk_cholesky_sync(void *stream, double *A, int n) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (ensure_status()) {
    ttk::set_error("ttk_cholesky_sync: status alloc failed");
    return TTK_ERR_HIP;
  }
  LinalgScope scope_(TTK_STREAM(stream), 4, n, n, n >= g_dense_block_min);
  if (n >= g_dense_block_min) {
    const int rc = ttk::cholesky_blocked(TTK_STREAM(stream), A, n, ttk::ctx().status);
    if (rc) return rc;
  } else {
    hipLaunchKernelGGL(chol_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), A, n, ttk::ctx().status);
    TTK_LAUNCH_CHECK();
  }
  int st = 0;
  TTK_HIP(hipMemcpyAsync(&st, ttk::ctx().status, sizeof(int), hipMemcpyDeviceToHost, TTK_STREAM(stream)));
  ttk::note_sync();
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  if (st) {
    ttk::set_error("%d-th leading minor of the array is not positive definite", st);
    return TTK_ERR_NOT_PD;
  }
  return TTK_OK;
}

int ttk_trsm_lower(void *stream, const double *L, int n, double *B, int nrhs, int ldb, int trans) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (n <= 0 || nrhs <= 0) return TTK_OK;
  if (n >= g_dense_block_min) return ttk::trsm_blocked(TTK_STREAM(stream), L, n, B, nrhs, ldb, trans);
  hipLaunchKernelGGL(trsm_kernel, dim3((nrhs + 63) / 64), dim3(256), 0, TTK_STREAM(stream), L, n, B, nrhs, ldb, trans);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_lu_sync(void *stream, double *A, int n, int *piv, double *work, double *rcond_out) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (ensure_status()) {
    ttk::set_error("ttk_lu_sync: status alloc failed");
    return TTK_ERR_HIP;
  }
  LinalgScope scope_(TTK_STREAM(stream), 3, n, n, n >= g_lu_block_min && n <= 7000);
  if (n >= g_lu_block_min && n <= 7000) {
    const int rc = ttk::lu_blocked(TTK_STREAM(stream), A, n, piv, work, ttk::ctx().status, ttk::ctx().rcond, 1);
    if (rc) return rc;
  } else {
    hipLaunchKernelGGL(lu_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), A, n, piv, work, ttk::ctx().status, ttk::ctx().rcond);
    TTK_LAUNCH_CHECK();
  }
  int st = 0;
  TTK_HIP(hipMemcpyAsync(&st, ttk::ctx().status, sizeof(int), hipMemcpyDeviceToHost, TTK_STREAM(stream)));
  TTK_HIP(hipMemcpyAsync(rcond_out, ttk::ctx().rcond, sizeof(double), hipMemcpyDeviceToHost, TTK_STREAM(stream)));
  ttk::note_sync();
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  if (st) {
    ttk::set_error("Matrix is singular (zero pivot at %d).", st);
    return TTK_ERR_SINGULAR;
  }
  return TTK_OK;
}

}  // extern "C"

namespace ttk {
int lu_factor_fork_rcond(hipStream_t st, double *A, int n, int *piv, double *work, int *forked) {
  *forked = 0;
  if (ensure_status()) {
    set_error("lu_factor_fork_rcond: status alloc failed");
    return TTK_ERR_HIP;
  }
  Ctx &c = ctx();
  LinalgScope scope_(st, 3, n, n, n >= g_lu_block_min && n <= 7000 ? 2 : 3);  // 2 forked dgecon, 3 one kernel
  if (!(n >= g_lu_block_min && n <= 7000)) {  // one-kernel getrf + dgecon (ttk_lu_sync's small path)
    hipLaunchKernelGGL(lu_kernel, dim3(1), dim3(1024), 0, st, A, n, piv, work, c.status, c.rcond);
    TTK_LAUNCH_CHECK();
    return TTK_OK;
  }
  // TTK_LU_FORK=0: the estimate on the caller's stream (same results; no second HW queue per process,
  // which matters when several solve processes share the GPU)
  static const int fork_on = getenv("TTK_LU_FORK") ? atoi(getenv("TTK_LU_FORK")) : 1;
  if (!fork_on) {
    const int rc = lu_blocked(st, A, n, piv, work, c.status, c.rcond, 1);
    return rc;
  }
  if (!c.side) {
    TTK_HIP(hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking));
    TTK_HIP(hipEventCreateWithFlags(&c.ev_fork, hipEventDisableTiming));
    TTK_HIP(hipEventCreateWithFlags(&c.ev_join, hipEventDisableTiming));
  }
  const int rc = lu_blocked(st, A, n, piv, work, c.status, c.rcond, 2);
  if (rc) return rc;
  TTK_HIP(hipEventRecord(c.ev_fork, st));
  TTK_HIP(hipStreamWaitEvent(c.side, c.ev_fork, 0));
  const int rr = lu_rcond_launch(c.side, A, n, piv, work, c.status, c.rcond);
  if (rr) return rr;
  TTK_HIP(hipEventRecord(c.ev_join, c.side));
  *forked = 1;
  return TTK_OK;
}

int lu_rcond_join(hipStream_t st) {
  TTK_HIP(hipStreamWaitEvent(st, ctx().ev_join, 0));
  return TTK_OK;
}
}  // namespace ttk

extern "C" {

int ttk_lu_solve(void *stream, const double *LU, int n, const int *piv, double *B, int nrhs, int ldb) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (n >= g_lu_block_min && n <= 12000 && nrhs <= 8 && nrhs > 0) return ttk::lu_solve_cols(TTK_STREAM(stream), LU, n, piv, B, nrhs, ldb);
  if (n <= 0 || nrhs <= 0) return TTK_OK;
  hipLaunchKernelGGL(lu_solve_kernel, dim3((nrhs + 63) / 64), dim3(256), 0, TTK_STREAM(stream), LU, n, piv, B, nrhs, ldb);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int64_t ttk_syev_work(int n) { return 2 * (int64_t)n * n + 2 * (n / 2 + 1) + 2 * (int64_t)n + 16; }

int ttk_syev(void *stream, double *A, int n, double *ev, double *W, double *work) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
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

int ttk_debug_counters(unsigned long long *out, int reset) {
  TTK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), sizeof(g_dbg)));
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    TTK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof(z)));
  }
  return TTK_OK;
}

static int g_syev_small = 1;

int ttk_syev_set_small(int on) {
  const int old = g_syev_small;
  g_syev_small = on;
  return old;
}

int64_t ttk_syev_extreme_work(int n) {
  if (n <= 0) return 0;
  const int64_t fused = (int64_t)n * n + 18 * (int64_t)n + 64;  // tri_step_kernel layout
  const int64_t need = syev_extreme_need(n);
  return need > fused ? need : fused;
}

static int g_syev_fused_max = TRI_FUSED_MAX;
static int g_syev_var = getenv("TTK_SYEV_VAR") ? atoi(getenv("TTK_SYEV_VAR")) : 12;  // syev_small_kernel variants
static int g_syev_small_wide = getenv("TTK_SYEV_WIDE") ? atoi(getenv("TTK_SYEV_WIDE")) : 64;  // 16-wave small kernel from this n
static int g_tri_rows = getenv("TTK_TRI_ROWS") ? atoi(getenv("TTK_TRI_ROWS")) : 4;  // largest n for the one-launch-per-step tridiagonalisation

int ttk_syev_set_fused_max(int n) {
  const int old = g_syev_fused_max;
  g_syev_fused_max = n < TRI_FUSED_MAX ? n : TRI_FUSED_MAX;
  return old;
}

int ttk_syev_extreme(void *stream, const double *A, int n, int which, double *ev, double *vec, double *work) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (n <= 0 || (which != 0 && which != 1)) {
    ttk::set_error("ttk_syev_extreme: bad arguments");
    return TTK_ERR_ARG;
  }
  const int64_t need = syev_extreme_need(n);
  const int use_lds = need <= LDS_DOUBLES;
  hipStream_t st = TTK_STREAM(stream);
  // path: 1 one launch per Householder step, 2 multi-workgroup, 3 small 1024, 4 small 256, 5 one kernel
  LinalgScope scope_(st, 2, n, which,
                     !use_lds && n > 2 ? (n <= g_syev_fused_max ? 1 : 2)
                     : (n >= 3 && n <= SYEV_SMALL_N && g_syev_small) ? (n >= g_syev_small_wide ? 3 : 4) : 5);
  if (!use_lds && n > 2 && n <= g_syev_fused_max) {  // one launch per Householder step
    double *Aw = work, *gv = work + (int64_t)n * n;
    double *dv = gv, *ov = dv + n, *tv = ov + 2 * n;  // layout of tri_finish_kernel: dv ov ev2 tv ...
    const int rb = g_tri_rows;  // rows per block (4 = one row per wave)
    const int nblk = (n + rb - 1) / rb;
    double *pvb = gv + 11 * (int64_t)n, *vbuf = pvb + 2 * (int64_t)n, *partb = vbuf + 2 * (int64_t)n;
    TTK_HIP(hipMemcpyAsync(Aw, A, sizeof(double) * (size_t)n * n, hipMemcpyDeviceToDevice, st));
    const int one_max = ttk::ctx().knob[TTK_KNOB_TRI_ONE];
    if (rb == 4 && n <= 513 && n <= one_max) {  // the whole tridiagonalisation in one workgroup
      const size_t shm = (size_t)(6 * n + 1) * sizeof(double);
      if (n <= 257)
        hipLaunchKernelGGL((tri_wg_kernel<4, 4>), dim3(1), dim3(1024), shm, st, Aw, n, tv, ov, dv, nblk);
      else
        hipLaunchKernelGGL((tri_wg_kernel<8, 1>), dim3(1), dim3(1024), shm, st, Aw, n, tv, ov, dv, nblk);
      TTK_LAUNCH_CHECK();
      return tri_finish_launch(st, Aw, n, which, gv, ev, vec);
    }
    const int hoist = rb == 4 && n <= 512 && ttk::ctx().knob[TTK_KNOB_TRI_HOIST] ? (n <= 256 ? 1 : 2) : 0;
    ttk::Ctx &cx = ttk::ctx();
    if (hoist && cx.knob[TTK_KNOB_TRI_PERSIST]) {  // every step in one launch (in-launch hand-offs)
      int rc = ttk::dep_counter(stream);
      if (rc != TTK_OK) return rc;
      const unsigned target = cx.dep_total, tick = cx.tick_total;
      cx.dep_total += (unsigned)nblk * (unsigned)(n - 2);
      cx.tick_total += (unsigned)nblk;
      if (hoist == 1)
        hipLaunchKernelGGL((tri_persist_kernel<1, 1, 4>), dim3(nblk), dim3(256), 0, st, Aw, n, tv, ov, dv, pvb, partb,
                           vbuf, nblk, cx.dep, target, tick);
      else
        hipLaunchKernelGGL((tri_persist_kernel<2, 2, 8>), dim3(nblk), dim3(256), 0, st, Aw, n, tv, ov, dv, pvb, partb,
                           vbuf, nblk, cx.dep, target, tick);
      hipLaunchKernelGGL(tri_tail_kernel, dim3(1), dim3(256), 0, st, Aw, n, tv, pvb, partb, vbuf, nblk);
      TTK_LAUNCH_CHECK();
      return tri_finish_launch(st, Aw, n, which, gv, ev, vec);
    }
    for (int k = 0; k + 2 < n; ++k) {
      if (hoist == 1)
        hipLaunchKernelGGL((tri_step_hoist_kernel<1, 1, 4>), dim3(nblk), dim3(256), 0, st, Aw, n, k, tv, ov, dv, pvb,
                           partb, vbuf, nblk);
      else if (hoist == 2)
        hipLaunchKernelGGL((tri_step_hoist_kernel<2, 2, 8>), dim3(nblk), dim3(256), 0, st, Aw, n, k, tv, ov, dv, pvb,
                           partb, vbuf, nblk);
      else
        hipLaunchKernelGGL(tri_step_kernel, dim3(nblk), dim3(256), 0, st, Aw, n, k, tv, ov, dv, pvb, partb, vbuf, nblk,
                           rb);
    }
    hipLaunchKernelGGL(tri_tail_kernel, dim3(1), dim3(256), 0, st, Aw, n, tv, pvb, partb, vbuf, nblk);
    TTK_LAUNCH_CHECK();
    return tri_finish_launch(st, Aw, n, which, gv, ev, vec);
  }
  if (!use_lds && n > 2) {  // multi-workgroup tridiagonalisation, one-workgroup finish
    double *Aw = work, *gv = work + (int64_t)n * n;
    double *dv = gv, *ov = dv + n, *tv = ov + 2 * n;  // layout of tri_finish_kernel: dv ov ev2 tv ...
    double *pv = gv + 11 * (int64_t)n, *partials = gv + 12 * (int64_t)n;
    const int nblk = (n + TRB - 1) / TRB;
    TTK_HIP(hipMemcpyAsync(Aw, A, sizeof(double) * (size_t)n * n, hipMemcpyDeviceToDevice, st));
    for (int k = 0; k + 2 < n; ++k) {
      hipLaunchKernelGGL(tri_update_kernel, dim3(nblk), dim3(256), 0, st, Aw, n, k, tv, ov, dv, pv, partials, nblk);
      hipLaunchKernelGGL(tri_matvec_kernel, dim3(nblk), dim3(256), 0, st, Aw, n, k, tv, pv, partials);
      TTK_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(tri_update_kernel, dim3(nblk), dim3(256), 0, st, Aw, n, n - 2, tv, ov, dv, pv, partials, nblk);
    TTK_LAUNCH_CHECK();
    return tri_finish_launch(st, Aw, n, which, gv, ev, vec);
  }
  if (n >= 3 && n <= SYEV_SMALL_N && g_syev_small) {
    const size_t shm_s = (size_t)syev_small_need(n) * sizeof(double);
    if (n >= g_syev_small_wide) {
      allow_big_lds(syev_small_kernel<1024>, shm_s);
      hipLaunchKernelGGL(syev_small_kernel<1024>, dim3(1), dim3(1024), shm_s, st, A, n, which, ev, vec, g_svd_timing,
                         g_syev_var);
    } else if (ttk::ctx().knob[TTK_KNOB_SYEV_WAVES8]) {
      allow_big_lds(syev_small_kernel<512, 2>, shm_s);
      hipLaunchKernelGGL((syev_small_kernel<512, 2>), dim3(1), dim3(512), shm_s, st, A, n, which, ev, vec,
                         g_svd_timing, g_syev_var);
    } else {
      allow_big_lds(syev_small_kernel<256>, shm_s);
      hipLaunchKernelGGL(syev_small_kernel<256>, dim3(1), dim3(256), shm_s, st, A, n, which, ev, vec, g_svd_timing,
                         g_syev_var);
    }
    TTK_LAUNCH_CHECK();
    return TTK_OK;
  }
  const size_t shm = use_lds ? need * sizeof(double) : 0;
  allow_big_lds(syev_extreme_kernel, shm);
  int nt = 4 * n;
  nt = nt < 64 ? 64 : (nt > 1024 ? 1024 : (nt + 63) / 64 * 64);
  hipLaunchKernelGGL(syev_extreme_kernel, dim3(1), dim3(nt), shm, TTK_STREAM(stream), A, n, which, ev, vec, work,
                     use_lds);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

}  // extern "C"
