// LGMRES (PETSc KSPLGMRES semantics) building blocks on the device.
//
// The Krylov basis V, the Hessenberg matrices and the Givens rotations stay in HBM/L2; the host
// only runs the integer bookkeeping of the restart/augmentation loop and reads ONE scalar
// (the new residual estimate) per Arnoldi step for the convergence test -- the same decision
// PETSc's KSPConvergedDefault takes (oracle/petsc_lgmres.py restates the algorithm).
//
// hh layout (doubles, ld = max_k+1):  HH[(max_k+2) x ld] | HES[(max_k+2) x ld] | GRS[max_k+2]
//                                     | CC[ld] | SS[ld] | status[8]
#include <math.h>

#include "ttk_common.h"
#include <vector>
#include "ttk_internal.h"

namespace {

struct HH {
  double *hh, *hes, *grs, *cc, *ss, *st;
  int ld;
  __device__ HH(double *base, int max_k) {
    ld = max_k + 1;
    hh = base;
    hes = hh + (max_k + 2) * ld;
    grs = hes + (max_k + 2) * ld;
    cc = grs + (max_k + 2);
    ss = cc + ld;
    st = ss + ld;
  }
};

// Speculative (host-sync-free) Arnoldi chunks: `Ctl` carries the stop flag ctl[0] and one record
// (step marker, res, hapend, null, HH(it,it)) per step of the chunk at ctl[1 + 5*slot].  Once a
// step meets a stop condition every later kernel of the chunk returns at entry, so the Hessenberg
// state stays exactly where the host-side loop stops.
struct Ctl {
  double *ctl;
  int slot;
  double marker, ttol, divtol;
};

__device__ inline bool ctl_stopped(const Ctl &c) { return c.ctl && c.ctl[0] != 0.0; }

__device__ inline void ctl_record(const Ctl &c, double res, bool hapend, bool null_flag, double diag) {
  if (!c.ctl) return;
  double *r = c.ctl + 1 + 5 * c.slot;
  r[0] = c.marker;
  r[1] = res;
  r[2] = hapend ? 1.0 : 0.0;
  r[3] = null_flag ? 1.0 : 0.0;
  r[4] = diag;
  // KSPConvergedDefault's tests (rtol/atol, divergence, non-finite) plus breakdown / null rotation
  if (hapend || null_flag || !(res == res) || isinf(res) || res <= c.ttol || res >= c.divtol) c.ctl[0] = 1.0;
}

constexpr int MAXV = 128;
struct PtrList {
  const double *p[MAXV];
};

// Hessenberg column `it` update: apply the previous Givens rotations, form the new one, update
// GRS.  `col` (LDS, it+2 entries) holds HH(0..it+1, it) on entry; the rotations are read into LDS
// first and the serial chain runs on LDS (not on dependent global loads), then the column is
// written back in parallel.  Returns (via the Ctl / st record) res, hapend, null, HH(it,it).
__device__ void hess_update(HH &H, int it, double *col, double *cs, double *sn, bool hapend, const Ctl &cl) {
  const int tid = threadIdx.x, nt = blockDim.x, ld = H.ld;
  for (int j = tid; j < it; j += nt) {
    cs[j] = H.cc[j];
    sn[j] = H.ss[j];
  }
  __syncthreads();
  if (tid == 0) {
    for (int j = 1; j <= it; ++j) {
      const double t0 = col[j - 1];
      const double t1 = col[j];
      col[j - 1] = cs[j - 1] * t0 + sn[j - 1] * t1;
      col[j] = cs[j - 1] * t1 - sn[j - 1] * t0;
    }
    double res = 0.0, null_flag = 0.0;
    if (!hapend) {
      const double hv = col[it], hv1 = col[it + 1];
      const double tr = sqrt(hv * hv + hv1 * hv1);
      if (tr == 0.0) {
        null_flag = 1.0;
      } else {
        H.cc[it] = hv / tr;
        H.ss[it] = hv1 / tr;
        H.grs[it + 1] = -(H.ss[it] * H.grs[it]);
        H.grs[it] = H.cc[it] * H.grs[it];
        col[it] = H.cc[it] * hv + H.ss[it] * hv1;
        res = fabs(H.grs[it + 1]);
      }
    }
    H.st[0] = res;
    H.st[1] = hapend ? 1.0 : 0.0;
    H.st[2] = null_flag;
    H.st[3] = col[it];
    ctl_record(cl, res, hapend, null_flag != 0.0, col[it]);
  }
  __syncthreads();
  for (int j = tid; j <= it + 1; j += nt) H.hh[j * ld + it] = col[j];
}


// KSPGMRESClassicalGramSchmidtOrthogonalization (REFINE_NEVER) + new HH/HES column +
// happy-breakdown test + KSPLGMRESUpdateHessenberg.  st[0]=res, st[1]=hapend, st[2]=null,
// st[3]=HH(it,it) after rotation.
__global__ __launch_bounds__(1024) void arnoldi_kernel(double *V, int n, int it, double *base, int max_k,
                                                       double haptol, Ctl cl) {
  if (ctl_stopped(cl)) return;
  __shared__ double h[MAXV + 2];
  __shared__ double red[16];
  HH H(base, max_k);
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  double *w = V + (int64_t)(it + 1) * n;
  // h_j = <V_j, w>, j = 0..it (one wave per j)
  for (int j = wid; j <= it; j += nw) {
    const double *vj = V + (int64_t)j * n;
    double s = ttk::chain_ahead<8>(
        ttk::steps_below(lane, n, 64), [&](int k) { return vj[lane + 64 * k]; }, [&](int k) { return w[lane + 64 * k]; },
        0.0);
    s = ttk::wave_sum(s);
    if (lane == 0) h[j] = s;
  }
  __syncthreads();
  // w -= sum_j h_j V_j
  for (int i = tid; i < n; i += nt)
    w[i] = ttk::chain_ahead<8, true>(
        it + 1, [&](int j) { return h[j]; }, [&](int j) { return V[(int64_t)j * n + i]; }, w[i]);
  __syncthreads();
  double s2 = ttk::chain_ahead<8>(
      ttk::steps_below(tid, n, nt), [&](int k) { return w[tid + nt * k]; }, [&](int k) { return w[tid + nt * k]; }, 0.0);
  s2 = ttk::block_sum(s2, red);
  const double tt = sqrt(s2);
  const int ld = H.ld;
  __shared__ double cs[MAXV + 2], sn[MAXV + 2];
  for (int j = tid; j <= it; j += nt) H.hes[j * ld + it] = h[j];
  double hapbnd = fabs(tt / H.grs[it]);
  if (hapbnd > haptol) hapbnd = haptol;
  const bool hapend = !(tt > hapbnd);
  if (!hapend) {
    const double inv = 1.0 / tt;
    for (int i = tid; i < n; i += nt) w[i] *= inv;
  }
  if (tid == 0) {
    H.hes[(it + 1) * ld + it] = tt;
    h[it + 1] = tt;
  }
  __syncthreads();
  hess_update(H, it, h, cs, sn, hapend, cl);
}

// KSPLGMRESBuildSoln's back substitution y = HH(0:it, 0:it) \ GRS in GRS, in its serial order, with
// the triangle and GRS staged in LDS first by the whole block (hl: (it+1)^2 doubles, ys: it+1): the
// dependent chain then waits on LDS loads instead of one L2 round trip per term (bit-identical)
__device__ void hh_backsub(HH &H, int it, double *hl, double *ys) {
  const int tid = threadIdx.x, nt = blockDim.x, ld = H.ld, w = it + 1;
  for (int e = tid; e < w * w; e += nt) {
    const int k = e / w, j = e - k * w;
    hl[e] = j >= k ? H.hh[k * ld + j] : 0.0;
  }
  for (int j = tid; j <= it; j += nt) ys[j] = H.grs[j];
  __syncthreads();
  if (tid == 0) {
    ys[it] = ys[it] / hl[it * w + it];
    for (int k = it - 1; k >= 0; --k) {
      double t0 = ys[k];
      for (int j = k + 1; j <= it; ++j) t0 -= hl[k * w + j] * ys[j];
      ys[k] = t0 / hl[k * w + k];
    }
  }
  __syncthreads();
  for (int j = tid; j <= it; j += nt) H.grs[j] = ys[j];
}

// avec = HES(0:it_total+1, 0:it_total) GRS: element jj sums its terms in the serial loop's order (ii
// ascending from max(jj-1, 0)), one thread per element
__device__ __forceinline__ void hes_times_grs(const HH &H, int it_total, double *avec) {
  const int ld = H.ld;
  for (int jj = threadIdx.x; jj <= it_total; jj += blockDim.x) {
    double a = 0.0;
    for (int ii = jj > 0 ? jj - 1 : 0; ii <= it_total; ++ii) a += H.hes[jj * ld + ii] * H.grs[ii];
    avec[jj] = a;
  }
}

// KSPLGMRESBuildSoln: back substitution in place in GRS, temp = sum y_j basis_j, x += temp.
__global__ __launch_bounds__(1024) void build_kernel(double *base, int max_k, int it, PtrList basis, int nvec,
                                                     int n, double *x, double *aug_temp) {
  extern __shared__ double hl[];  // (it+1)^2 triangle
  __shared__ double y[MAXV + 2];
  HH H(base, max_k);
  const int tid = threadIdx.x, nt = blockDim.x;
  hh_backsub(H, it, hl, y);
  for (int i = tid; i < n; i += nt) {
    const double t = ttk::chain_ahead<8>(
        nvec, [&](int j) { return y[j]; }, [&](int j) { return basis.p[j][i]; }, 0.0);
    aug_temp[i] = t;
    x[i] += t;
  }
}

// A*aug = V (HES y) / ||aug_temp||, augvec = aug_temp / ||aug_temp||
__global__ __launch_bounds__(1024) void aug_kernel(const double *base_c, int max_k, int it_total, const double *V,
                                                   int n, const double *aug_temp, double *augvec, double *a_augvec) {
  __shared__ double avec[MAXV + 2];
  __shared__ double red[16];
  HH H(const_cast<double *>(base_c), max_k);
  const int ld = H.ld;
  const int tid = threadIdx.x, nt = blockDim.x;
  hes_times_grs(H, it_total, avec);
  double s2 = ttk::chain_ahead<8>(
      ttk::steps_below(tid, n, nt), [&](int k) { return aug_temp[tid + nt * k]; },
      [&](int k) { return aug_temp[tid + nt * k]; }, 0.0);
  s2 = ttk::block_sum(s2, red);
  const double inv = 1.0 / sqrt(s2);
  for (int i = tid; i < n; i += nt) {
    augvec[i] = aug_temp[i] * inv;
    const double t = ttk::chain_ahead<8>(
        it_total + 1, [&](int j) { return avec[j]; }, [&](int j) { return V[(int64_t)j * n + i]; }, 0.0);
    a_augvec[i] = t * inv;
  }
}

// ---------------------------------------------------------------- multi-workgroup variants
// One workgroup streams the whole basis (it+1 vectors of length n, twice per Arnoldi step) through
// a single CU; for the long local vectors of the iterative solves (3m ~ 1e4-3e4 doubles, restart
// up to 100, i.e. tens of MB per step) that is bandwidth-bound at one CU's share of L2.  These
// split the same classical Gram-Schmidt over the chip: (1) per (vector j, chunk) partial dots,
// (2) per chunk: h_j = sum of partials (fixed order), w -= sum_j h_j V_j, partial |w|^2,
// (3) one workgroup: |w|, breakdown test, w /= |w|, Hessenberg + Givens update.  Every reduction
// runs in a fixed order, so results are deterministic run to run.
constexpr int ARN_CHUNK = 2048;  // elements of one (j, chunk) partial dot
constexpr int ARN_UPD = 512;     // elements per update block

__global__ __launch_bounds__(256) void arnoldi_dot_kernel(const double *__restrict__ V, int n, int it,
                                                          double *__restrict__ partials, int nchunk, Ctl cl) {
  if (ctl_stopped(cl)) return;
  __shared__ double red[16];
  const int c = blockIdx.x, j = blockIdx.y, tid = threadIdx.x;
  const double *vj = V + (int64_t)j * n, *w = V + (int64_t)(it + 1) * n;
  const int i0 = c * ARN_CHUNK, i1 = i0 + ARN_CHUNK < n ? i0 + ARN_CHUNK : n;
  double s = ttk::chain_ahead<8>(
      ttk::steps_below(i0 + tid, i1, 256), [&](int k) { return vj[i0 + tid + 256 * k]; },
      [&](int k) { return w[i0 + tid + 256 * k]; }, 0.0);
  s = ttk::block_sum(s, red);
  if (tid == 0) partials[(int64_t)j * nchunk + c] = s;
}

__global__ __launch_bounds__(256) void arnoldi_update_kernel(double *__restrict__ V, int n, int it,
                                                             const double *__restrict__ partials, int nchunk,
                                                             double *__restrict__ normpart, double *base,
                                                             int max_k, Ctl cl) {
  if (ctl_stopped(cl)) return;
  __shared__ double h[MAXV + 2];
  __shared__ double red[16];
  const int tid = threadIdx.x;
  for (int j = tid; j <= it; j += 256)
    h[j] = ttk::sum_ahead<8>(nchunk, [&](int c) { return partials[(int64_t)j * nchunk + c]; }, 0.0);
  __syncthreads();
  if (blockIdx.x == 0) {
    HH H(base, max_k);
    for (int j = tid; j <= it; j += 256) {
      H.hh[j * H.ld + it] = h[j];
      H.hes[j * H.ld + it] = h[j];
    }
  }
  double *w = V + (int64_t)(it + 1) * n;
  const int i = blockIdx.x * ARN_UPD + tid;
  double s2 = 0.0;
  for (int ii = i; ii < n && ii < (blockIdx.x + 1) * ARN_UPD; ii += 256) {
    const double acc = ttk::chain_ahead<8, true>(
        it + 1, [&](int j) { return h[j]; }, [&](int j) { return V[(int64_t)j * n + ii]; }, w[ii]);
    w[ii] = acc;
    s2 = fma(acc, acc, s2);
  }
  s2 = ttk::block_sum(s2, red);
  if (tid == 0) normpart[blockIdx.x] = s2;
}

__global__ __launch_bounds__(1024) void arnoldi_finish_kernel(double *V, int n, int it, const double *normpart,
                                                              int nblk, double *base, int max_k, double haptol,
                                                              Ctl cl) {
  if (ctl_stopped(cl)) return;
  __shared__ double s_tt;
  HH H(base, max_k);
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) {
    s_tt = sqrt(ttk::sum_ahead<8>(nblk, [&](int b) { return normpart[b]; }, 0.0));
  }
  __syncthreads();
  const double tt = s_tt;
  const int ld = H.ld;
  __shared__ double col[MAXV + 2], cs[MAXV + 2], sn[MAXV + 2];
  for (int j = tid; j <= it; j += nt) col[j] = H.hh[j * ld + it];  // h_j from arnoldi_update_kernel
  double hapbnd = fabs(tt / H.grs[it]);
  if (hapbnd > haptol) hapbnd = haptol;
  const bool hapend = !(tt > hapbnd);
  double *w = V + (int64_t)(it + 1) * n;
  if (!hapend) {
    const double inv = 1.0 / tt;
    for (int i = tid; i < n; i += nt) w[i] *= inv;
  }
  if (tid == 0) {
    H.hes[(it + 1) * ld + it] = tt;
    col[it + 1] = tt;
  }
  __syncthreads();
  hess_update(H, it, col, cs, sn, hapend, cl);
}

// The three kernels above as ONE launch (in-launch hand-offs, ttk_common.h): blocks
// [0, ndot) are the (chunk, vector) partial dots, [ndot, ndot + nblk) the update blocks, the last
// block the finish.  Every role runs the same arithmetic as its kernel above with 256 threads (the
// finish's reductions are serial or elementwise, so its thread count never changes a bit); the
// words one role hands to the next in this launch (partials, w, the norm parts, the HH column) go
// out with sc1 stores and come in with sc1 loads.  Stopped chunks still arrive, so the counter
// stays in step with the host's targets.
__global__ __launch_bounds__(256) void arnoldi_fused_kernel(double *__restrict__ V, int n, int it,
                                                            double *__restrict__ partials, int nchunk,
                                                            double *__restrict__ normpart, int nblk, double *base,
                                                            int max_k, double haptol, Ctl cl, unsigned *dep,
                                                            unsigned t_dots, unsigned t_upd, unsigned tick_base) {
  __shared__ double h[MAXV + 2];
  __shared__ double red[16];
  const bool stopped = ctl_stopped(cl);
  // roles by start order (ttk::ticket): the dot blocks first, the finish last -- every wait is on
  // workgroups that are already running
  const int tid = threadIdx.x, b = ttk::ticket(dep, tick_base);
  const int ndot = nchunk * (it + 1);
  double *w = V + (int64_t)(it + 1) * n;
  if (b < ndot) {  // arnoldi_dot_kernel
    if (!stopped) {
      const int c = b % nchunk, j = b / nchunk;
      const double *vj = V + (int64_t)j * n;
      const int i0 = c * ARN_CHUNK, i1 = i0 + ARN_CHUNK < n ? i0 + ARN_CHUNK : n;
      double acc = ttk::chain_ahead<8>(
          ttk::steps_below(i0 + tid, i1, 256), [&](int k) { return vj[i0 + tid + 256 * k]; },
          [&](int k) { return w[i0 + tid + 256 * k]; }, 0.0);
      acc = ttk::block_sum(acc, red);
      if (tid == 0) ttk::st_sc1(partials + (int64_t)j * nchunk + c, acc);
    }
    ttk::dep_arrive(dep);
    return;
  }
  if (b < ndot + nblk) {  // arnoldi_update_kernel
    const int blk = b - ndot;
    ttk::dep_wait(dep, t_dots);
    __syncthreads();
    if (!stopped) {
      for (int j = tid; j <= it; j += 256)
        h[j] = ttk::sum_ahead<8>(nchunk, [&](int c) { return ttk::ld_sc1(partials + (int64_t)j * nchunk + c); }, 0.0);
      __syncthreads();
      if (blk == 0) {
        HH H(base, max_k);
        for (int j = tid; j <= it; j += 256) {
          ttk::st_sc1(H.hh + j * H.ld + it, h[j]);
          H.hes[j * H.ld + it] = h[j];
        }
      }
      double s2 = 0.0;
      for (int ii = blk * ARN_UPD + tid; ii < n && ii < (blk + 1) * ARN_UPD; ii += 256) {
        const double acc = ttk::chain_ahead<8, true>(
            it + 1, [&](int j) { return h[j]; }, [&](int j) { return V[(int64_t)j * n + ii]; }, w[ii]);
        ttk::st_sc1(w + ii, acc);
        s2 = fma(acc, acc, s2);
      }
      s2 = ttk::block_sum(s2, red);
      if (tid == 0) ttk::st_sc1(normpart + blk, s2);
    }
    ttk::dep_arrive(dep);
    return;
  }
  // arnoldi_finish_kernel
  ttk::dep_wait(dep, t_upd);
  __syncthreads();
  if (stopped) return;
  __shared__ double s_tt;
  HH H(base, max_k);
  if (tid == 0) s_tt = sqrt(ttk::sum_ahead<8>(nblk, [&](int q) { return ttk::ld_sc1(normpart + q); }, 0.0));
  __syncthreads();
  const double tt = s_tt;
  const int ld = H.ld;
  __shared__ double col[MAXV + 2], cs[MAXV + 2], sn[MAXV + 2];
  for (int j = tid; j <= it; j += 256) col[j] = ttk::ld_sc1(H.hh + j * ld + it);
  double hapbnd = fabs(tt / H.grs[it]);
  if (hapbnd > haptol) hapbnd = haptol;
  const bool hapend = !(tt > hapbnd);
  if (!hapend) {
    const double inv = 1.0 / tt;
    for (int i = tid; i < n; i += 256) w[i] = ttk::ld_sc1(w + i) * inv;
  }
  if (tid == 0) {
    H.hes[(it + 1) * ld + it] = tt;
    col[it + 1] = tt;
  }
  __syncthreads();
  hess_update(H, it, col, cs, sn, hapend, cl);
}

// y = HH \ GRS (back substitution in GRS), once, by a single thread (it <= 100)
__global__ __launch_bounds__(256) void build_solve_kernel(double *base, int max_k, int it) {
  extern __shared__ double hl[];
  __shared__ double ys[MAXV + 2];
  HH H(base, max_k);
  hh_backsub(H, it, hl, ys);
}

// temp = sum_j y_j basis_j, x += temp (chunks over the chip; y = GRS after build_solve_kernel)
__global__ __launch_bounds__(256) void build_axpy_kernel(const double *base, int max_k, PtrList basis, int nvec,
                                                         int n, double *x, double *aug_temp) {
  __shared__ double y[MAXV + 2];
  HH H(const_cast<double *>(base), max_k);
  for (int j = threadIdx.x; j < nvec; j += 256) y[j] = H.grs[j];
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double t = 0.0;
  for (int j = 0; j < nvec; ++j) t += y[j] * basis.p[j][i];
  aug_temp[i] = t;
  x[i] += t;
}

// partial |aug_temp|^2 per block
__global__ __launch_bounds__(256) void sumsq_part_kernel(const double *__restrict__ a, int n, double *part) {
  __shared__ double red[16];
  const int i0 = blockIdx.x * ARN_UPD;
  double s2 = 0.0;
  for (int i = i0 + threadIdx.x; i < n && i < i0 + ARN_UPD; i += 256) s2 = fma(a[i], a[i], s2);
  s2 = ttk::block_sum(s2, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s2;
}

// augvec = aug_temp / |aug_temp|, A*aug = V (HES GRS) / |aug_temp|
__global__ __launch_bounds__(256) void aug_apply_kernel(const double *base_c, int max_k, int it_total,
                                                        const double *V, int n, const double *aug_temp,
                                                        const double *part, int nblk, double *augvec,
                                                        double *a_augvec) {
  __shared__ double avec[MAXV + 2];
  __shared__ double s_inv;
  HH H(const_cast<double *>(base_c), max_k);
  const int ld = H.ld, tid = threadIdx.x;
  hes_times_grs(H, it_total, avec);
  if (tid == 0) {
    double s2 = 0.0;
    for (int b = 0; b < nblk; ++b) s2 += part[b];
    s_inv = 1.0 / sqrt(s2);
  }
  __syncthreads();
  const int i = blockIdx.x * 256 + tid;
  if (i >= n) return;
  const double inv = s_inv;
  augvec[i] = aug_temp[i] * inv;
  double t = 0.0;
  for (int j = 0; j <= it_total; ++j) t += avec[j] * V[(int64_t)j * n + i];
  a_augvec[i] = t * inv;
}

double *lgmres_scratch(int64_t n) {  // partials / norm parts of the current context (grown, never shrunk)
  ttk::Ctx &c = ttk::ctx();
  if (n > c.lgmres_n) {
    if (c.lgmres) {
      (void)(c.stream ? hipStreamSynchronize(c.stream) : hipDeviceSynchronize());
      (void)hipFree(c.lgmres);
    }
    const int64_t want = n < 65536 ? 65536 : n;
    if (hipMalloc(reinterpret_cast<void **>(&c.lgmres), want * sizeof(double)) != hipSuccess) {
      c.lgmres = nullptr;
      c.lgmres_n = 0;
      return nullptr;
    }
    c.lgmres_n = want;
  }
  return c.lgmres;
}

}  // namespace

int ttk::presize_lgmres() { return lgmres_scratch(1) ? TTK_OK : TTK_ERR_HIP; }  // see ttk::presize_splitk

namespace {

// (it+1)*n at or above which the multi-workgroup kernels run: per-context knob
static inline int64_t mw_min() { return ttk::ctx().knob[TTK_KNOB_LGMRES_MW_MIN]; }

}  // namespace

extern "C" {

}  // extern "C"

static int arnoldi_launch(hipStream_t st_, double *V, int n, int it, double *hh, int max_k, double haptol,
                          const Ctl &cl, const char *who) {
  if (it + 1 > MAXV || max_k + 2 > MAXV + 2) {
    ttk::set_error("%s: restart %d too large (max %d)", who, max_k, MAXV);
    return TTK_ERR_ARG;
  }
  if ((int64_t)(it + 1) * n >= mw_min()) {
    const int nchunk = (n + ARN_CHUNK - 1) / ARN_CHUNK, nblk = (n + ARN_UPD - 1) / ARN_UPD;
    double *partials = lgmres_scratch((int64_t)(it + 1) * nchunk + nblk + 64);
    if (!partials) {
      ttk::set_error("%s: scratch allocation failed", who);
      return TTK_ERR_HIP;
    }
    double *normpart = partials + (int64_t)(it + 1) * nchunk;
    ttk::Ctx &cx = ttk::ctx();
    if (cx.knob[TTK_KNOB_ARNOLDI_ONE]) {  // one launch: dots -> update -> finish over hand-offs
      if (int rc = ttk::dep_counter(st_)) return rc;
      const unsigned ndot = (unsigned)(nchunk * (it + 1));
      const unsigned t_dots = cx.dep_total + ndot, t_upd = t_dots + (unsigned)nblk;
      cx.dep_total = t_upd;
      const unsigned tick = cx.tick_total;
      cx.tick_total += ndot + (unsigned)nblk + 1u;
      hipLaunchKernelGGL(arnoldi_fused_kernel, dim3(ndot + nblk + 1), dim3(256), 0, st_, V, n, it, partials, nchunk,
                         normpart, nblk, hh, max_k, haptol, cl, cx.dep, t_dots, t_upd, tick);
      TTK_LAUNCH_CHECK();
      return TTK_OK;
    }
    hipLaunchKernelGGL(arnoldi_dot_kernel, dim3(nchunk, it + 1), dim3(256), 0, st_, V, n, it, partials, nchunk, cl);
    hipLaunchKernelGGL(arnoldi_update_kernel, dim3(nblk), dim3(256), 0, st_, V, n, it, partials, nchunk, normpart,
                       hh, max_k, cl);
    hipLaunchKernelGGL(arnoldi_finish_kernel, dim3(1), dim3(1024), 0, st_, V, n, it, normpart, nblk, hh, max_k,
                       haptol, cl);
    TTK_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(arnoldi_kernel, dim3(1), dim3(1024), 0, st_, V, n, it, hh, max_k, haptol, cl);
    TTK_LAUNCH_CHECK();
  }
  return TTK_OK;
}

extern "C" {

int ttk_lgmres_arnoldi_sync(void *stream, double *V, int n, int it, double *hh, int max_k, double haptol,
                            double *res_out, int *hapend_out) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  const Ctl none{nullptr, 0, 0.0, 0.0, 0.0};
  int rc = arnoldi_launch(TTK_STREAM(stream), V, n, it, hh, max_k, haptol, none, "ttk_lgmres_arnoldi_sync");
  if (rc) return rc;
  const int ld = max_k + 1;
  const int64_t st_off = 2 * (int64_t)(max_k + 2) * ld + (max_k + 2) + 2 * ld;
  double st[4];
  rc = ttk_read_sync(stream, hh + st_off, st, 4);
  if (rc) return rc;
  res_out[0] = st[0];
  res_out[1] = st[3];
  hapend_out[0] = (int)st[1];
  hapend_out[1] = (int)st[2];
  return TTK_OK;
}

int ttk_lgmres_arnoldi_async(void *stream, double *V, int n, int it, double *hh, int max_k, double haptol,
                             double ttol, double divtol, double *ctl, int slot, double marker) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  const Ctl cl{ctl, slot, marker, ttol, divtol};
  return arnoldi_launch(TTK_STREAM(stream), V, n, it, hh, max_k, haptol, cl, "ttk_lgmres_arnoldi_async");
}

int ttk_lgmres_chunk(void *stream, int64_t schur, double *V, int n, int it0, int k, double *hh, int max_k,
                     double haptol, double ttol, double divtol, double *ctl, double marker0) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  for (int q = 0; q < k; ++q) {
    const int it = it0 + q;
    int rc = ttk::schur_apply(stream, schur, V + (int64_t)it * n, V + (int64_t)(it + 1) * n);
    if (rc) return rc;
    rc = ttk_lgmres_arnoldi_async(stream, V, n, it, hh, max_k, haptol, ttol, divtol, ctl, q, marker0 + q);
    if (rc) return rc;
  }
  return TTK_OK;
}

int ttk_lgmres_build(void *stream, double *hh, int max_k, int it, const double *const *basis, int nvec, int n,
                     double *x, double *aug_temp) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (nvec > MAXV || it + 1 > MAXV) {
    ttk::set_error("ttk_lgmres_build: too many basis vectors %d", nvec);
    return TTK_ERR_ARG;
  }
  PtrList pl;
  for (int j = 0; j < nvec; ++j) pl.p[j] = basis[j];
  if ((int64_t)nvec * n >= mw_min()) {
    const size_t shm = (size_t)(it + 1) * (it + 1) * sizeof(double);
    if (shm > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void *>(build_solve_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipLaunchKernelGGL(build_solve_kernel, dim3(1), dim3(256), shm, TTK_STREAM(stream), hh, max_k, it);
    hipLaunchKernelGGL(build_axpy_kernel, dim3((n + 255) / 256), dim3(256), 0, TTK_STREAM(stream), hh, max_k, pl,
                       nvec, n, x, aug_temp);
  } else {
    const size_t shm = (size_t)(it + 1) * (it + 1) * sizeof(double);
    if (shm > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void *>(build_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipLaunchKernelGGL(build_kernel, dim3(1), dim3(1024), shm, TTK_STREAM(stream), hh, max_k, it, pl, nvec, n, x,
                       aug_temp);
  }
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_lgmres_aug(void *stream, const double *hh, int max_k, int it_total, const double *V, int n,
                   double inv_nrm_unused, const double *aug_temp, double *augvec, double *a_augvec) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  (void)inv_nrm_unused;
  if (it_total + 1 > MAXV) {
    ttk::set_error("ttk_lgmres_aug: it_total %d too large", it_total);
    return TTK_ERR_ARG;
  }
  if ((int64_t)(it_total + 1) * n >= mw_min()) {
    const int nblk = (n + ARN_UPD - 1) / ARN_UPD;
    double *part = lgmres_scratch(nblk + 64);
    if (!part) {
      ttk::set_error("ttk_lgmres_aug: scratch allocation failed");
      return TTK_ERR_HIP;
    }
    hipLaunchKernelGGL(sumsq_part_kernel, dim3(nblk), dim3(256), 0, TTK_STREAM(stream), aug_temp, n, part);
    hipLaunchKernelGGL(aug_apply_kernel, dim3((n + 255) / 256), dim3(256), 0, TTK_STREAM(stream), hh, max_k, it_total,
                       V, n, aug_temp, part, nblk, augvec, a_augvec);
  } else {
    hipLaunchKernelGGL(aug_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), hh, max_k, it_total, V, n, aug_temp,
                       augvec, a_augvec);
  }
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

// ---------------------------------------------------------------- whole LGMRES solve (one call)
// PETSc KSPLGMRES (`src/tt_ipm.py:101-162`; restated in oracle/petsc_lgmres.py) on a Schur operator
// handle: the host bookkeeping of tensor-train-interior-point-method_amd/lgmres.py (restart cycles,
// augmentation order, KSPConvergedDefault replayed on the speculative chunks' records) in C++, so a
// local KKT solve is one library call.  The kernel sequence is that of the Python driver with the
// native operator, hence the iterates are bit-identical to it.
namespace {

int64_t hh_size(int max_k) {
  const int64_t ld = max_k + 1;
  return 2 * (int64_t)(max_k + 2) * ld + (max_k + 2) + 2 * ld + 8;
}

int lg_converged(int k, double rnorm, double rtol, double abstol, double dtol, double &rnorm0, double &ttol) {
  if (k == 0) {
    rnorm0 = rnorm;
    ttol = fmax(rtol * rnorm, abstol);
  }
  if (rnorm != rnorm || isinf(rnorm)) return -9;             // DIVERGED_NANORINF
  if (rnorm <= ttol) return rnorm < abstol ? 3 : 2;           // CONVERGED_ATOL / _RTOL
  if (rnorm >= dtol * rnorm0) return -4;                      // DIVERGED_DTOL
  return 0;
}

}  // namespace

int ttk_lgmres(ttk_ctx ctx, int64_t schur, const double *b, double *x, int64_t n64, int restart, int augment,
               double rtol, int max_it, int chunk, ttk_lgmres_info *info) {
  ttk::CtxScope scope(ctx);
  ttk::Ctx &cx = ttk::ctx();
  void *stream = reinterpret_cast<void *>(cx.stream);
  const int n = (int)n64;
  const int max_k = restart, aug_dim = augment;
  const double abstol = 1e-50, dtol = 1e5, haptol = 1e-30;
  const int nd = aug_dim > 1 ? aug_dim : 1;
  chunk = chunk > 0 ? chunk : 1;
  if (n <= 0 || max_k < 1 || max_k + 1 > MAXV) {
    ttk::set_error("ttk_lgmres: bad size n=%d restart=%d", n, max_k);
    return TTK_ERR_ARG;
  }
  // workspace: V | hh | augvecs | a_augvecs | aug_temp | ctl
  const int64_t nV = (int64_t)(max_k + 1) * n, nH = hh_size(max_k), nA = (int64_t)nd * n, nC = 1 + 5 * (int64_t)chunk;
  const int64_t need = nV + nH + 2 * nA + n + nC + 64;
  // the scratch base holds the multi-workgroup Arnoldi / augmentation partials (arnoldi_launch,
  // ttk_lgmres_aug: (it+1)*ceil(n/ARN_CHUNK) + ceil(n/ARN_UPD) + 64 doubles at most); the solve's
  // workspace starts after that slab so the partials can never overwrite V
  const int64_t slab0 = (int64_t)(max_k + 2) * ((n + ARN_CHUNK - 1) / ARN_CHUNK) + (n + ARN_UPD - 1) / ARN_UPD + 64;
  const int64_t slab = slab0 > 65536 ? slab0 : 65536;
  double *ws = lgmres_scratch(need + 1 + slab);
  if (!ws) {
    ttk::set_error("ttk_lgmres: workspace allocation failed");
    return TTK_ERR_HIP;
  }
  ws += slab;
  double *V = ws, *hh = V + nV, *augvecs = hh + nH, *a_augvecs = augvecs + nA, *aug_temp = a_augvecs + nA,
         *ctl = aug_temp + n;
  const int64_t grs_off = 2 * (int64_t)(max_k + 2) * (max_k + 1);
  int rc;
  if ((rc = ttk_fill(stream, x, n, 0.0)) || (rc = ttk_fill(stream, hh, nH, 0.0)) || (rc = ttk_fill(stream, ctl, nC, 0.0)))
    return rc;
  std::vector<int64_t> aug_order(nd, 0);
  int aug_ct = 0, its = 0, itcount = 0, reason = 0, nmv = 0;
  bool guess_zero = true;
  double res = 0.0, rnorm0 = 0.0, ttol = 0.0;
  const int64_t one_shape[1] = {n}, unit[1] = {1};
  auto copy = [&](double *dst, const double *src, double al, double be) {
    return ttk_copy_nd(stream, src, dst, 1, one_shape, unit, unit, al, be);
  };
  auto norm = [&](const double *v, double &out) {
    double d = 0.0;
    int r = ttk_dot_nd_sync(stream, v, v, 1, one_shape, unit, unit, &d);
    out = sqrt(fmax(d, 0.0));
    return r;
  };
  int it_arnoldi = max_k - aug_dim;
  auto matvec_or_aug = [&](int li) {
    if (li < it_arnoldi) return ttk::schur_apply(stream, schur, V + (int64_t)li * n, V + (int64_t)(li + 1) * n);
    const int64_t order = li - it_arnoldi + 1;
    int spot = 0;
    for (int ii = 0; ii < aug_dim; ++ii)
      if (aug_order[ii] == order) {
        spot = ii;
        break;
      }
    return copy(V + (int64_t)(li + 1) * n, a_augvecs + (int64_t)spot * n, 1.0, 0.0);
  };
  while (!reason) {
    if (guess_zero) {
      if ((rc = copy(V, b, 1.0, 0.0))) return rc;
    } else {
      if ((rc = ttk::schur_apply(stream, schur, x, V))) return rc;
      ++nmv;
      if ((rc = copy(V, b, 1.0, -1.0))) return rc;  // r = b - A x
    }
    it_arnoldi = max_k - aug_dim;
    const int it_total = it_arnoldi + aug_ct;
    if ((rc = norm(V, res))) return rc;
    if ((rc = ttk_fill(stream, hh + grs_off, 1, res))) return rc;
    if (res == 0.0) {
      reason = 3;
      break;
    }
    if ((rc = copy(V, V, 1.0 / res, 0.0))) return rc;
    reason = lg_converged(its, res, rtol, abstol, dtol, rnorm0, ttol);
    int loc_it = 0;
    bool hapend = false;
    double last_diag = 1.0;
    while (!reason && loc_it < it_total && its < max_it) {
      int kmax = chunk;
      if (it_total - loc_it < kmax) kmax = it_total - loc_it;
      if (max_it - its < kmax) kmax = max_it - its;
      double recs[5 * 64 + 1];
      int nrec;
      if (kmax <= 1) {
        if ((rc = matvec_or_aug(loc_it))) return rc;
        double rb[2];
        int fl[2];
        if ((rc = ttk_lgmres_arnoldi_sync(stream, V, n, loc_it, hh, max_k, haptol, rb, fl))) return rc;
        recs[0] = its + 1;
        recs[1] = rb[0];
        recs[2] = fl[0];
        recs[3] = fl[1];
        recs[4] = rb[1];
        nrec = 1;
      } else {
        if (kmax > 64) kmax = 64;
        const double divtol = dtol * rnorm0;
        const bool in_native = loc_it + kmax <= it_arnoldi;
        if (in_native) {
          if ((rc = ttk_lgmres_chunk(stream, schur, V, n, loc_it, kmax, hh, max_k, haptol, ttol, divtol, ctl,
                                     (double)(its + 1))))
            return rc;
        } else {
          for (int q = 0; q < kmax; ++q) {
            if ((rc = matvec_or_aug(loc_it + q))) return rc;
            if ((rc = ttk_lgmres_arnoldi_async(stream, V, n, loc_it + q, hh, max_k, haptol, ttol, divtol, ctl, q,
                                               (double)(its + q + 1))))
              return rc;
          }
        }
        double h[1 + 5 * 64];
        if ((rc = ttk_read_sync(stream, ctl, h, 1 + 5 * kmax))) return rc;
        for (int q = 0; q < 5 * kmax; ++q) recs[q] = h[1 + q];
        nrec = kmax;
      }
      for (int q = 0; q < nrec; ++q) {
        const double *r = recs + 5 * q;
        if (r[0] != its + 1) {
          ttk::set_error("ttk_lgmres: device stopped the Arnoldi chunk at step %d without a host-side stop reason",
                         its);
          return TTK_ERR_ARG;
        }
        hapend = r[2] != 0.0;
        if (r[3] != 0.0) {
          reason = -2;  // DIVERGED_NULL
          break;
        }
        res = r[1];
        last_diag = r[4];
        nmv += loc_it < it_arnoldi;
        ++loc_it;
        ++its;
        reason = lg_converged(its, res, rtol, abstol, dtol, rnorm0, ttol);
        if (hapend && !reason) {
          reason = -5;  // DIVERGED_BREAKDOWN
          break;
        }
        if (reason) break;
      }
      if (reason == -2 || reason == -5) break;
    }
    const int cycle_its = loc_it;
    const int it = loc_it - 1;
    bool built = false;
    if (it >= 0) {
      int ita = max_k - aug_dim, it_aug;
      if (ita >= it + 1) {
        it_aug = 0;
        ita = it + 1;
      } else {
        it_aug = (it + 1) - ita;
      }
      if (last_diag == 0.0) {
        ttk::set_error("ttk_lgmres: HH(it,it) is identically zero; it = %d (PETSC_ERR_CONV_FAILED)", it);
        return TTK_ERR_NOT_CONVERGED;
      }
      std::vector<const double *> ptrs;
      for (int j = 0; j < ita; ++j) ptrs.push_back(V + (int64_t)j * n);
      for (int ii = 0; ii < it_aug; ++ii) {
        int spot = 0;
        for (int jj = 0; jj < aug_dim; ++jj)
          if (aug_order[jj] == ii + 1) {
            spot = jj;
            break;
          }
        ptrs.push_back(augvecs + (int64_t)spot * n);
      }
      if ((rc = ttk_lgmres_build(stream, hh, max_k, it, ptrs.data(), (int)ptrs.size(), n, x, aug_temp))) return rc;
      built = true;
    }
    if (!reason && its < max_it && aug_dim > 0 && built) {
      int spot = 0;
      if (aug_ct == 0) {
        spot = 0;
        ++aug_ct;
      } else if (aug_ct < aug_dim) {
        spot = aug_ct;
        ++aug_ct;
      } else {
        spot = 0;
        for (int ii = 0; ii < aug_dim; ++ii)
          if (aug_order[ii] == aug_dim) spot = ii;
      }
      for (int ii = 0; ii < aug_dim; ++ii) aug_order[ii] += 1;
      aug_order[spot] = 1;
      if ((rc = ttk_lgmres_aug(stream, hh, max_k, it_total, V, n, 0.0, aug_temp, augvecs + (int64_t)spot * n,
                               a_augvecs + (int64_t)spot * n)))
        return rc;
    }
    itcount += cycle_its;
    if (itcount >= max_it) {
      if (!reason) reason = -3;  // DIVERGED_ITS
      break;
    }
    guess_zero = false;
  }
  if (info) {
    info->reason = reason;
    info->its = its;
    info->res = res;
    info->matvecs = nmv;
  }
  return TTK_OK;
}

int ttk_lgmres_set_mw_threshold(int elems) {
  int &k = ttk::ctx().knob[TTK_KNOB_LGMRES_MW_MIN];
  const int old = k;
  k = elems;
  return old;
}

}  // extern "C"
