// Core-contraction kernel: one pairwise step of a planned einsum as an offset-table GEMM on
// fp64 MFMA (v_mfma_f64_16x16x4_f64).
//
//   C[b,m,n] = alpha * sum_k A[a_b[b]+a_m[m]+a_k[k]] * B[b_b[b]+b_k[k]+b_n[n]] + beta * C[...]
//
// Offset tables (int64, device) make any strided / permuted operand layout free: the TT-core
// contractions of the hot path ('lsr,lML,sMNS,rNR->LSR', 'lsr,smnS,LSR,rnR->lmL', ...) are
// executed as 2-3 of these steps with no transpose copies (the reference pays explicit
// transpose-copies between its dgemms, cy_src/lgmres_cy.pyx:56-120).
//
// Tile: 32x32 outputs per 256-thread workgroup = 2x2 waves, each wave one 16x16 MFMA tile.
// K is staged through LDS 16 at a time (4 MFMAs per wave per stage).  f64 MFMA lane maps
// (MI355X guide §3): A[i=l&15][k=l>>4], B[k=l>>4][j=l&15], D: col=l&15, row=(l>>4)+4*r.
#include <hip/hip_ext.h>

#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "ttk_common.h"
#include "ttk_internal.h"

namespace {

constexpr int TM = 32, TN = 32, TK = 16;

struct GemmArgs {
  const double *A;
  const double *B;
  double *C;
  const int64_t *offs;
  int nb, M, N, K;
  double alpha, beta;
};

struct GroupPtrs {
  const double *const *A;
  const double *const *B;
  double *const *C;
};

typedef double double4_t __attribute__((ext_vector_type(4)));

// One 32x32 output tile over the K range [kb, ke), staged TS = 64 K values per LDS stage (4x fewer
// barrier / global-latency rounds than one 16-K stage).  Software pipeline: the offset-table
// entries of stage s+2 and the operands of stage s+1 are in flight while stage s's MFMAs run, so
// the gather's two dependent global loads (table entry, then operand) are each hidden behind a
// stage of compute.  The MFMA sequence per output tile is k = kb, kb+4, ... in order, exactly as
// with 16-K stages (trailing all-zero K groups are skipped), so results are unchanged bit for bit.
// out != nullptr: raw partial sums (no alpha/beta) to a dense [M][N] slab (split-K);
// out == nullptr: alpha/beta epilogue into C through the output offset tables.
// SC1: the partial sums go out with write-through (sc1) stores, for a consumer on another CU.
template <int TS, bool SC1 = false>  // K per LDS stage (16 / 32 / 64: picked per launch from K; LDS 8.4 / 17 / 34 KB)
__device__ __forceinline__ void gemm_tile(const double *__restrict__ A, const double *__restrict__ B,
                                          double *__restrict__ C, const int64_t *__restrict__ offs,
                                          int nb, int M, int N, int K, double alpha, double beta,
                                          int b, int m0, int n0, int kb, int ke, double *__restrict__ out) {
  constexpr int TQ = TS / 8, RP = 256 / TS;  // staged elements per thread per operand; rows per pass
  __shared__ double As[TS][TM + 1];
  __shared__ double Bs[TS][TN + 1];
  const int64_t *a_b = offs;
  const int64_t *a_m = a_b + nb;
  const int64_t *a_k = a_m + M;
  const int64_t *b_b = a_k + K;
  const int64_t *b_k = b_b + nb;
  const int64_t *b_n = b_k + K;
  const int64_t *c_b = b_n + N;
  const int64_t *c_m = c_b + nb;
  const int64_t *c_n = c_m + M;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t abase = a_b[b], bbase = b_b[b];
  // Staging map per operand, picked from its offset tables (uniform per workgroup): element q of a
  // thread is (row r0 + q*dr, k k0 + kq + q*dk).  Row-major staging (lanes along m|n, the K runs
  // of 8 spread over the waves) unless the operand is contiguous along K but not along m|n; then
  // lanes run along K (TS consecutive k, 256/TS rows per pass), so a wave load covers contiguous
  // runs of K instead of 32 rows' worth of scattered lines.
  const bool a_kmaj = K > 1 && a_k[1] - a_k[0] == 1 && !(M > 1 && a_m[1] - a_m[0] == 1);
  const bool b_kmaj = K > 1 && b_k[1] - b_k[0] == 1 && !(N > 1 && b_n[1] - b_n[0] == 1);
  const int ar0 = a_kmaj ? tid / TS : tid & 31, adr = a_kmaj ? RP : 0;
  const int akq = a_kmaj ? tid % TS : tid >> 5, adk = a_kmaj ? 0 : 8;
  const int br0 = b_kmaj ? tid / TS : tid & 31, bdr = b_kmaj ? RP : 0;
  const int bkq = b_kmaj ? tid % TS : tid >> 5, bdk = b_kmaj ? 0 : 8;
  int64_t arow[TQ], brow[TQ];
  unsigned aok = 0, bok = 0;  // row-valid bits
#pragma unroll
  for (int q = 0; q < TQ; ++q) {
    const int m = m0 + ar0 + q * adr, n = n0 + br0 + q * bdr;
    arow[q] = abase + (m < M ? a_m[m] : 0);
    brow[q] = bbase + (n < N ? b_n[n] : 0);
    aok |= (m < M ? 1u : 0u) << q;
    bok |= (n < N ? 1u : 0u) << q;
  }
  int64_t oa[TQ], ob[TQ];
  double ra[TQ], rb[TQ];
  auto fetch_offs = [&](int k0) {
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const int ka = k0 + akq + q * adk, kb_ = k0 + bkq + q * bdk;
      oa[q] = ka < ke ? a_k[ka] : 0;
      ob[q] = kb_ < ke ? b_k[kb_] : 0;
    }
  };
  auto fetch_vals = [&](int k0) {
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const bool oka = ((aok >> q) & 1u) && k0 + akq + q * adk < ke;
      const bool okb = ((bok >> q) & 1u) && k0 + bkq + q * bdk < ke;
      ra[q] = oka ? A[arow[q] + oa[q]] : 0.0;
      rb[q] = okb ? B[brow[q] + ob[q]] : 0.0;
    }
  };
  double4_t acc = {0.0, 0.0, 0.0, 0.0};
  if (kb < ke) {
    fetch_offs(kb);
    fetch_vals(kb);
    if (kb + TS < ke) fetch_offs(kb + TS);
  }
  for (int k0 = kb; k0 < ke; k0 += TS) {
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      As[akq + q * adk][ar0 + q * adr] = ra[q];
      Bs[bkq + q * bdk][br0 + q * bdr] = rb[q];
    }
    __syncthreads();
    if (k0 + TS < ke) {
      fetch_vals(k0 + TS);
      if (k0 + 2 * TS < ke) fetch_offs(k0 + 2 * TS);
    }
    const int ns = (ke - k0 + 3) >> 2;  // K groups of 4 with data in this stage
#pragma unroll
    for (int s = 0; s < TS / 4; ++s) {
      if (s < ns) {
        const double a = As[s * 4 + (lane >> 4)][wr * 16 + (lane & 15)];
        const double bv = Bs[s * 4 + (lane >> 4)][wc * 16 + (lane & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv, acc, 0, 0, 0);
      }
    }
    __syncthreads();
  }
  const int col = n0 + wc * 16 + (lane & 15);
  if (col >= N) return;
  if (out) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wr * 16 + (lane >> 4) + 4 * r;
      if (row < M) {
        if (SC1)
          ttk::st_sc1(out + (int64_t)row * N + col, acc[r]);
        else
          out[(int64_t)row * N + col] = acc[r];
      }
    }
    return;
  }
  const int64_t cb = c_b[b] + c_n[col];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m0 + wr * 16 + (lane >> 4) + 4 * r;
    if (row < M) {
      double *p = C + cb + c_m[row];
      const double v = alpha * acc[r];
      *p = (beta == 0.0) ? v : v + beta * (*p);
    }
  }
}

// Throughput variant for large steps (dense Schur GEMMs, graphm-sized contractions): 64x64 outputs
// per workgroup, each wave a 32x32 block as 2x2 MFMA tiles (4 accumulators: 16 MFMAs per LDS
// stage instead of 4).  Same K order per output element as gemm_tile, so results are identical.
constexpr int BM = 64, BN = 64;

template <int KS>
__global__ __launch_bounds__(256) void gemm_offs64_kernel(GemmArgs g) {
  constexpr int NQ = KS / 4;  // staged elements per thread per operand
  __shared__ double As[KS][BM + 1];
  __shared__ double Bs[KS][BN + 1];
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM, b = blockIdx.z;
  const int M = g.M, N = g.N, K = g.K, nb = g.nb;
  const int64_t *a_b = g.offs;
  const int64_t *a_m = a_b + nb;
  const int64_t *a_k = a_m + M;
  const int64_t *b_b = a_k + K;
  const int64_t *b_k = b_b + nb;
  const int64_t *b_n = b_k + K;
  const int64_t *c_b = b_n + N;
  const int64_t *c_m = c_b + nb;
  const int64_t *c_n = c_m + M;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  // staging map per operand as in gemm_tile: element q = (row r0 + q*dr, k kq + q*dk); row-major
  // (lanes along m|n, k = tid/64 + 4q) unless the operand is contiguous along K only, then lanes
  // run along K (KS consecutive k, 256/KS rows per pass)
  constexpr int RP = 256 / KS;
  const bool a_kmaj = K > 1 && a_k[1] - a_k[0] == 1 && !(M > 1 && a_m[1] - a_m[0] == 1);
  const bool b_kmaj = K > 1 && b_k[1] - b_k[0] == 1 && !(N > 1 && b_n[1] - b_n[0] == 1);
  const int ar0 = a_kmaj ? tid / KS : tid & 63, adr = a_kmaj ? RP : 0;
  const int akq = a_kmaj ? tid % KS : tid >> 6, adk = a_kmaj ? 0 : 4;
  const int br0 = b_kmaj ? tid / KS : tid & 63, bdr = b_kmaj ? RP : 0;
  const int bkq = b_kmaj ? tid % KS : tid >> 6, bdk = b_kmaj ? 0 : 4;
  const int64_t abase = a_b[b], bbase = b_b[b];
  int64_t arow[NQ], brow[NQ];
  unsigned aok = 0, bok = 0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int m = m0 + ar0 + q * adr, n = n0 + br0 + q * bdr;
    arow[q] = abase + (m < M ? a_m[m] : 0);
    brow[q] = bbase + (n < N ? b_n[n] : 0);
    aok |= (m < M ? 1u : 0u) << q;
    bok |= (n < N ? 1u : 0u) << q;
  }
  int64_t oa[NQ], ob[NQ];
  double ra[NQ], rb[NQ];
  auto fetch_offs = [&](int k0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int ka = k0 + akq + q * adk, kb_ = k0 + bkq + q * bdk;
      oa[q] = ka < K ? a_k[ka] : 0;
      ob[q] = kb_ < K ? b_k[kb_] : 0;
    }
  };
  auto fetch = [&](int k0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool oka = ((aok >> q) & 1u) && k0 + akq + q * adk < K;
      const bool okb = ((bok >> q) & 1u) && k0 + bkq + q * bdk < K;
      ra[q] = oka ? g.A[arow[q] + oa[q]] : 0.0;
      rb[q] = okb ? g.B[brow[q] + ob[q]] : 0.0;
    }
  };
  double4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = double4_t{0.0, 0.0, 0.0, 0.0};
  fetch_offs(0);
  fetch(0);
  if (KS < K) fetch_offs(KS);
  for (int k0 = 0; k0 < K; k0 += KS) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      As[akq + q * adk][ar0 + q * adr] = ra[q];
      Bs[bkq + q * bdk][br0 + q * bdr] = rb[q];
    }
    __syncthreads();
    if (k0 + KS < K) {
      fetch(k0 + KS);
      if (k0 + 2 * KS < K) fetch_offs(k0 + 2 * KS);
    }
#pragma unroll
    for (int s = 0; s < KS / 4; ++s) {
      const int kr = s * 4 + (lane >> 4);
      const double a0 = As[kr][wr * 32 + (lane & 15)], a1 = As[kr][wr * 32 + 16 + (lane & 15)];
      const double b0 = Bs[kr][wc * 32 + (lane & 15)], b1 = Bs[kr][wc * 32 + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wc * 32 + j * 16 + (lane & 15);
    if (col >= N) continue;
    const int64_t cb = c_b[b] + c_n[col];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wr * 32 + i * 16 + (lane >> 4) + 4 * r;
        if (row < M) {
          double *p = g.C + cb + c_m[row];
          const double v = g.alpha * acc[i][j][r];
          *p = (g.beta == 0.0) ? v : v + g.beta * (*p);
        }
      }
  }
}

template <int TS>
__global__ __launch_bounds__(256) void gemm_offs_kernel(GemmArgs g) {
  const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM, b = blockIdx.z;
  gemm_tile<TS>(g.A, g.B, g.C, g.offs, g.nb, g.M, g.N, g.K, g.alpha, g.beta, b, m0, n0, 0, g.K, nullptr);
}

// split-K: blockIdx.z = b * nsplit + split; partial tile sums to part[split][b][M][N]
template <int TS>
__global__ __launch_bounds__(256) void gemm_offs_splitk_kernel(GemmArgs g, int nsplit, int kc, double *part) {
  const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM;
  const int b = blockIdx.z / nsplit, sp = blockIdx.z % nsplit;
  const int kb = sp * kc, ke = kb + kc < g.K ? kb + kc : g.K;
  double *out = part + ((int64_t)sp * g.nb + b) * g.M * g.N;
  gemm_tile<TS>(g.A, g.B, g.C, g.offs, g.nb, g.M, g.N, g.K, g.alpha, g.beta, b, m0, n0, kb, ke, out);
}

// Split-K in ONE launch: the split blocks of a tile store their partial tiles write-through (sc1),
// drain, and count their arrival on the tile's counter with an agent-scope release (sc1 stores +
// s_waitcnt vmcnt(0) + workgroup barrier + release fence + one atomic add; the last arriver runs an
// agent acquire and loads sc1 -- ttk_common.h, memory model).  The block whose arrival completes the count sums the tile's partials
// in split order and writes C -- the reduce kernel's arithmetic below, element for element -- and
// resets the counter for the next launch.  Nobody waits: a block that is not last just exits, so
// the grid drains whatever the residency.
template <int TS>
__global__ __launch_bounds__(256) void gemm_offs_splitk_fused_kernel(GemmArgs g, int nsplit, int kc, double *part,
                                                                     unsigned *cnt) {
  __shared__ unsigned s_old;
  const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM;
  const int b = blockIdx.z / nsplit, sp = blockIdx.z % nsplit;
  const int kb = sp * kc, ke = kb + kc < g.K ? kb + kc : g.K;
  const int64_t mn = (int64_t)g.M * g.N;
  gemm_tile<TS, true>(g.A, g.B, g.C, g.offs, g.nb, g.M, g.N, g.K, g.alpha, g.beta, b, m0, n0, kb, ke,
                      part + ((int64_t)sp * g.nb + b) * mn);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned *c = cnt + ((int64_t)b * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  if (threadIdx.x == 0) {  // ttk_common.h, memory model
#ifndef TTK_HANDOFF_RELAXED
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    s_old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (s_old != (unsigned)(nsplit - 1)) return;
#ifndef TTK_HANDOFF_RELAXED
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
  const int64_t *a_b = g.offs;
  const int64_t *c_b = a_b + g.nb + g.M + g.K + g.nb + g.K + g.N;
  const int64_t *c_m = c_b + g.nb;
  const int64_t *c_n = c_m + g.M;
  // each thread owns EPT tile elements; the partials are loaded U splits at a time for all of them
  // before any is added (sc1 loads in flight together), then added in split order per element
  constexpr int EPT = TM * TN / 256, U = 8;
  const int64_t slab = (int64_t)g.nb * mn;
  const double *base = part + (int64_t)b * mn;
  int64_t r[EPT];
  bool ok[EPT];
  double acc[EPT];
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    const int e = threadIdx.x + q * 256, row = m0 + e / TN, col = n0 + e % TN;
    ok[q] = row < g.M && col < g.N;
    r[q] = ok[q] ? (int64_t)row * g.N + col : 0;
    acc[q] = 0.0;
  }
  for (int s0 = 0; s0 < nsplit; s0 += U) {
    double v[EPT][U];
#pragma unroll
    for (int q = 0; q < EPT; ++q)
#pragma unroll
      for (int u = 0; u < U; ++u) v[q][u] = (ok[q] && s0 + u < nsplit) ? ttk::ld_sc1(base + (s0 + u) * slab + r[q]) : 0.0;
#pragma unroll
    for (int q = 0; q < EPT; ++q)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (s0 + u < nsplit) acc[q] += v[q][u];
  }
#pragma unroll
  for (int q = 0; q < EPT; ++q) {
    if (!ok[q]) continue;
    const int e = threadIdx.x + q * 256, row = m0 + e / TN, col = n0 + e % TN;
    double *p = g.C + c_b[b] + c_m[row] + c_n[col];
    const double v = g.alpha * acc[q];
    *p = (g.beta == 0.0) ? v : v + g.beta * (*p);
  }
  if (threadIdx.x == 0) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// C = alpha * sum_split part + beta * C (fixed summation order: deterministic)
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(GemmArgs g, int nsplit, const double *part) {
  const int64_t mn = (int64_t)g.M * g.N;
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= mn * g.nb) return;
  const int b = (int)(e / mn);
  const int64_t r = e - b * mn;
  const int row = (int)(r / g.N), col = (int)(r - (int64_t)row * g.N);
  double acc = 0.0;
  for (int sp = 0; sp < nsplit; ++sp) acc += part[((int64_t)sp * g.nb + b) * mn + r];
  const int64_t *a_b = g.offs;
  const int64_t *c_b = a_b + g.nb + g.M + g.K + g.nb + g.K + g.N;
  const int64_t *c_m = c_b + g.nb;
  const int64_t *c_n = c_m + g.M;
  double *p = g.C + c_b[b] + c_m[row] + c_n[col];
  const double v = g.alpha * acc;
  *p = (g.beta == 0.0) ? v : v + g.beta * (*p);
}

template <int TS>
__global__ __launch_bounds__(256) void gemm_offs_grouped_kernel(GemmArgs g, GroupPtrs p) {
  const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM;
  const int grp = blockIdx.z / g.nb, b = blockIdx.z % g.nb;
  gemm_tile<TS>(p.A[grp], p.B[grp], p.C[grp], g.offs, g.nb, g.M, g.N, g.K, g.alpha, g.beta, b, m0, n0, 0, g.K,
            nullptr);
}

// K per LDS stage for a launch: short contractions keep the small LDS footprint (occupancy hides
// the gather latency), long ones take fewer, deeper stages.  Any choice gives the same results.
static inline int stage_k(int K) { return K < 32 ? 16 : (K < 128 ? 32 : 64); }

// Independent problems of one einsum batch level in ONE launch: workgroup -> (problem, tile) through
// the tile prefix; each tile runs gemm_tile exactly as gemm_offs_kernel would (same n/m/b tile
// coordinates, same K order), so results are bit-identical to one launch per problem.
constexpr int GROUP_MAX = 24;
struct GemmGroup {
  GemmArgs p[GROUP_MAX];
  int tile0[GROUP_MAX + 1];
  int n;
};

template <int TS>
__global__ __launch_bounds__(256) void gemm_offs_group_kernel(GemmGroup G) {
  const int bid = blockIdx.x;
  int p = 0;
  while (p + 1 < G.n && bid >= G.tile0[p + 1]) ++p;
  const GemmArgs &g = G.p[p];
  int t = bid - G.tile0[p];
  const int ntn = (g.N + TN - 1) / TN, ntm = (g.M + TM - 1) / TM;
  const int n0 = (t % ntn) * TN;
  t /= ntn;
  const int m0 = (t % ntm) * TM;
  const int b = t / ntm;
  gemm_tile<TS>(g.A, g.B, g.C, g.offs, g.nb, g.M, g.N, g.K, g.alpha, g.beta, b, m0, n0, 0, g.K, nullptr);
}

// ------------------------------------------------------------------ element-wise (N-D strided)
__device__ __forceinline__ void nd_offsets(const ttk::NdDesc &d, int64_t lin, int64_t &o0,
                                           int64_t &o1, int64_t &o2) {
  o0 = o1 = o2 = 0;
  for (int i = d.ndim - 1; i >= 0; --i) {
    const int64_t e = d.shape[i];
    const int64_t q = lin / e;
    const int64_t r = lin - q * e;
    lin = q;
    o0 += r * d.s0[i];
    o1 += r * d.s1[i];
    o2 += r * d.s2[i];
  }
}

// several contiguous copies in one launch (ttk_copy_many): segment j owns flat indices
// [off[j], off[j+1]); exact copies
struct CopyMany {
  static constexpr int MAXN = 32;
  const double *src[MAXN];
  double *dst[MAXN];
  int64_t off[MAXN + 1];
  int n;
};

__global__ void copy_many_kernel(CopyMany m) {
  const int64_t total = m.off[m.n], stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    int j = 0;
    while (e >= m.off[j + 1]) ++j;
    m.dst[j][e - m.off[j]] = m.src[j][e - m.off[j]];
  }
}

__global__ void copy_nd_kernel(const double *__restrict__ src, double *__restrict__ dst,
                               ttk::NdDesc d, double alpha, double beta) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < d.total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t os, od, unused;
    nd_offsets(d, i, os, od, unused);
    const double v = alpha * src[os];
    dst[od] = (beta == 0.0) ? v : v + beta * dst[od];
  }
}

__global__ void mul_nd_kernel(const double *__restrict__ s1, const double *__restrict__ s2,
                              double *__restrict__ dst, ttk::NdDesc d, double alpha, double beta) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < d.total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t o1, o2, od;
    nd_offsets(d, i, o1, o2, od);
    const double v = alpha * s1[o1] * s2[o2];
    dst[od] = (beta == 0.0) ? v : v + beta * dst[od];
  }
}

// dst = alpha * src + beta * (gamma * src2), written in copy_nd_kernel's form so that it rounds like
// the two-step dev.scaled(src2, gamma) + dev.copy_(dst, src, alpha, beta) it replaces
__global__ void axpby_nd_kernel(const double *__restrict__ src, const double *__restrict__ src2,
                                double *__restrict__ dst, ttk::NdDesc d, double alpha, double beta, double gamma) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < d.total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t o1, o2, od;
    nd_offsets(d, i, o1, o2, od);
    const double t = gamma * src2[o2];
    const double v = alpha * src[o1];
    dst[od] = (beta == 0.0) ? v : v + beta * t;
  }
}

// TT-core assembly of the rank-additive sum (tt_add, cy_src/tt_ops_cy.pyx:228-258) in one launch:
// out (ro, mid, Ro) from contiguous a (ra, mid, Ra) and b (rb, mid, Rb).
//   mode 0: block diagonal (ro = ra + rb, Ro = Ra + Rb, zeros elsewhere)
//   mode 1: concatenation along the last axis (ro = ra = rb, Ro = Ra + Rb)
//   mode 2: concatenation along the first axis (ro = ra + rb, Ro = Ra = Rb)
__global__ void tt_join_kernel(const double *__restrict__ a, const double *__restrict__ b, double *__restrict__ out,
                               int ra, int Ra, int rb, int Rb, int64_t mid, int mode) {
  const int ro = mode == 1 ? ra : ra + rb, Ro = mode == 2 ? Ra : Ra + Rb;
  const int64_t total = (int64_t)ro * mid * Ro;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(e % Ro);
    const int64_t t = e / Ro;
    const int64_t m = t % mid;
    const int i = (int)(t / mid);
    double v = 0.0;
    if (mode == 0) {
      if (i < ra && j < Ra) v = a[((int64_t)i * mid + m) * Ra + j];
      else if (i >= ra && j >= Ra) v = b[((int64_t)(i - ra) * mid + m) * Rb + (j - Ra)];
    } else if (mode == 1) {
      v = j < Ra ? a[((int64_t)i * mid + m) * Ra + j] : b[((int64_t)i * mid + m) * Rb + (j - Ra)];
    } else {
      v = i < ra ? a[((int64_t)i * mid + m) * Ra + j] : b[((int64_t)(i - ra) * mid + m) * Rb + j];
    }
    out[e] = v;
  }
}

struct AxisScales {
  double v[16];
};

// dst = src * scale[coordinate along `axis`] (per-block column scaling of the AMEn sweep)
__global__ void scale_axis_kernel(const double *__restrict__ src, double *__restrict__ dst, ttk::NdDesc d, int axis,
                                  AxisScales sc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < d.total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t lin = i, os = 0, od = 0, ca = 0;
    for (int k = d.ndim - 1; k >= 0; --k) {
      const int64_t e = d.shape[k];
      const int64_t q = lin / e;
      const int64_t r = lin - q * e;
      lin = q;
      os += r * d.s0[k];
      od += r * d.s1[k];
      if (k == axis) ca = r;
    }
    dst[od] = src[os] * sc.v[ca];
  }
}

// the same scaling with per-block scales derived on the device from block sums of squares:
// sc = max(sqrt(ss), 1e-10) (np.maximum(np.sqrt(ss), 1e-10)), factor sc or 1.0 / sc
__global__ void scale_axis_ss_kernel(const double *__restrict__ src, double *__restrict__ dst, ttk::NdDesc d,
                                     int axis, const double *__restrict__ ss, int invert) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < d.total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t lin = i, os = 0, od = 0, ca = 0;
    for (int k = d.ndim - 1; k >= 0; --k) {
      const int64_t e = d.shape[k];
      const int64_t q = lin / e;
      const int64_t r = lin - q * e;
      lin = q;
      os += r * d.s0[k];
      od += r * d.s1[k];
      if (k == axis) ca = r;
    }
    const double nr = sqrt(ss[ca]);
    const double sc = nr > 1e-10 ? nr : 1e-10;
    dst[od] = src[os] * (invert ? 1.0 / sc : sc);
  }
}

__global__ void recip_kernel(const double *__restrict__ src, double *__restrict__ dst, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = 1.0 / src[i];
}

__global__ void fill_kernel(double *dst, int64_t n, double v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = v;
}

__global__ void add_diag_kernel(double *A, int n, int lda, double v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) A[(int64_t)i * lda + i] += v;
}

// out = x / ||x|| without a host round trip: the sum of squares is formed exactly as dot_nd_kernel
// forms <x, x> (same thread map and block reduction), then the host formula of dev.norm and
// dev.scaled (sqrt(max(s, 0)), 1.0 / nrm, alpha * x), so results are bit-identical to the synced path
__global__ void normalize_kernel(const double *__restrict__ x, ttk::NdDesc d, double *__restrict__ out) {
  __shared__ double red[16];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < d.total; i += blockDim.x) {
    int64_t ox, oy, unused;
    nd_offsets(d, i, ox, oy, unused);
    acc += x[ox] * x[oy];
  }
  acc = ttk::block_sum(acc, red);
  const double m = (0.0 > acc) ? 0.0 : acc;
  const double inv = 1.0 / sqrt(m);
  for (int64_t i = threadIdx.x; i < d.total; i += blockDim.x) {
    int64_t ox, oy, od;
    nd_offsets(d, i, ox, oy, od);
    out[od] = inv * x[ox];
  }
}

// Rayleigh tail of the step-size local solve: ev = <v, Mv>; Mv <- Mv - ev v; res2 = <Mv, Mv>
// (contiguous vectors, one workgroup; the operations and their order of dot_nd / copy_nd)
__global__ void rayleigh_tail_kernel(const double *__restrict__ v, double *__restrict__ Mv, int64_t n,
                                     double *__restrict__ out2, double beta) {
  __shared__ double red[16];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) acc += v[i] * Mv[i];
  const double ev = ttk::block_sum(acc, red);
  const double a = -ev;
  double acc2 = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double vv = a * v[i];  // written as copy_nd_kernel writes it (same contraction by the compiler)
    const double w = (beta == 0.0) ? vv : vv + beta * Mv[i];
    Mv[i] = w;
    acc2 += w * w;
  }
  acc2 = ttk::block_sum(acc2, red);
  if (threadIdx.x == 0) {
    out2[0] = ev;
    out2[1] = acc2;
  }
}

__global__ void dot_nd_kernel(const double *__restrict__ x, const double *__restrict__ y, ttk::NdDesc d,
                              double *out) {
  __shared__ double red[16];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < d.total; i += blockDim.x) {
    int64_t ox, oy, unused;
    nd_offsets(d, i, ox, oy, unused);
    acc += x[ox] * y[oy];
  }
  acc = ttk::block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = acc;
}

// The AMEn rank loop's residual updates (`src/tt_als.py:338-346`, `:466-472`): for q = 0..nq-1 in
// order, res <- -1 * neg_q + res (copy_nd_kernel's operations with alpha = -1, beta = 1), then
// <res, res> (dot_nd_kernel's thread map and block reduction) into out[q] -- every candidate rank's
// residual norm in one launch and one host read, bit-identical to the one-candidate-at-a-time loop.
__global__ __launch_bounds__(1024) void rank_scan_kernel(double *__restrict__ res, const double *__restrict__ negs,
                                                         int64_t n, int nq, double *__restrict__ out) {
  __shared__ double red[16];
  for (int q = 0; q < nq; ++q) {
    const double *ng = negs + (int64_t)q * n;
    double acc = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
      const double v = -1.0 * ng[i];
      const double w = v + 1.0 * res[i];
      res[i] = w;
      acc += w * w;
    }
    acc = ttk::block_sum(acc, red);
    if (threadIdx.x == 0) out[q] = acc;
  }
}

__global__ void sumsq_batched_kernel(const double *__restrict__ x, int64_t n, int64_t bstride, double *out) {
  __shared__ double red[16];
  const double *xb = x + blockIdx.x * bstride;
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) acc += xb[i] * xb[i];
  acc = ttk::block_sum(acc, red);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// the same sums over a strided batch: element i of batch b at x[b*bstride + (i/inner)*ostride + i%inner]
// (each batch = an (outer, inner) slab), summed in i order by the same threads as sumsq_batched_kernel
__global__ void sumsq_batched2_kernel(const double *__restrict__ x, int64_t n, int64_t bstride, int64_t inner,
                                      int64_t ostride, double *out) {
  __shared__ double red[16];
  const double *xb = x + blockIdx.x * bstride;
  double acc = 0.0;
  int64_t o = threadIdx.x / inner, r = threadIdx.x - o * inner;
  const int64_t so = blockDim.x / inner, sr = blockDim.x - so * inner;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double v = xb[o * ostride + r];
    acc += v * v;
    o += so;
    r += sr;
    if (r >= inner) {
      r -= inner;
      ++o;
    }
  }
  acc = ttk::block_sum(acc, red);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

int make_nd(ttk::NdDesc &d, int ndim, const int64_t *shape, const int64_t *s0, const int64_t *s1,
            const int64_t *s2) {
  if (ndim < 0 || ndim > ttk::MAXD) {
    ttk::set_error("ndim %d out of range (max %d)", ndim, ttk::MAXD);
    return TTK_ERR_ARG;
  }
  d.ndim = ndim;
  d.total = 1;
  for (int i = 0; i < ndim; ++i) {
    d.shape[i] = shape[i];
    d.s0[i] = s0 ? s0[i] : 0;
    d.s1[i] = s1 ? s1[i] : 0;
    d.s2[i] = s2 ? s2[i] : 0;
    d.total *= shape[i];
  }
  return TTK_OK;
}

inline int grid_for(int64_t n, int block) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return static_cast<int>(g);
}


// Contraction-kernel accounting (bench.py roofline): algorithmic FLOPs (2*M*N*K per GEMM step,
// the opt_einsum convention of SURVEY.md 8(d)) are always counted; with timing on, every
// contraction launch is bracketed by two HIP events on its own stream and the durations are
// summed at harvest (auto-harvest every EV_CHUNK events keeps the pool bounded).  The events are
// handed to hipExtLaunchKernelGGL, so they time the dispatch itself (no marker packets between).
struct ContractStats {
  double flops = 0.0, timed_flops = 0.0, timed_ms = 0.0;
  long long launches = 0, timed_launches = 0;
  bool timing = false;
  std::vector<hipEvent_t> ev;
  size_t used = 0;
};
ContractStats g_cs;
constexpr size_t EV_CHUNK = 8192;

int harvest_events() {
  if (g_cs.used == 0) return TTK_OK;
  TTK_HIP(hipEventSynchronize(g_cs.ev[g_cs.used - 1]));
  for (size_t i = 0; i + 1 < g_cs.used; i += 2) {
    float ms = 0.0f;
    TTK_HIP(hipEventElapsedTime(&ms, g_cs.ev[i], g_cs.ev[i + 1]));
    g_cs.timed_ms += ms;
  }
  g_cs.used = 0;
  return TTK_OK;
}

// start/stop events for the next contraction launch (nullptr when timing is off); they are
// passed to hipExtLaunchKernelGGL, which records them with the dispatch itself
int contract_events(hipEvent_t *ev0, hipEvent_t *ev1) {
  *ev0 = *ev1 = nullptr;
  if (!g_cs.timing) return TTK_OK;
  if (g_cs.used + 2 > EV_CHUNK) {
    int rc = harvest_events();
    if (rc != TTK_OK) return rc;
  }
  while (g_cs.ev.size() < g_cs.used + 2) {
    hipEvent_t e;
    TTK_HIP(hipEventCreate(&e));
    g_cs.ev.push_back(e);
  }
  *ev0 = g_cs.ev[g_cs.used];
  *ev1 = g_cs.ev[g_cs.used + 1];
  g_cs.used += 2;
  return TTK_OK;
}

void contract_count(double flops) {
  g_cs.flops += flops;
  g_cs.launches += 1;
  if (g_cs.timing) {
    g_cs.timed_flops += flops;
    g_cs.timed_launches += 1;
  }
}

}  // namespace

namespace ttk {
// contraction accounting for kernels launched outside this file (fused local apply)
int contract_events_ext(hipEvent_t *ev0, hipEvent_t *ev1) { return contract_events(ev0, ev1); }
void contract_count_ext(double flops) { contract_count(flops); }
}  // namespace ttk

extern "C" {

}  // extern "C"

namespace {
// split-K on/off and K per split: per-context knobs (TTK_KNOB_SPLITK / _SPLITK_MINK)
static inline bool splitk_on() { return ttk::ctx().knob[TTK_KNOB_SPLITK] != 0; }
constexpr int SPLITK_TILES_MAX = 256;  // split-K runs only when the tile grid is below 256 tiles
static inline int splitk_mink() {
  const int k = ttk::ctx().knob[TTK_KNOB_SPLITK_MINK];
  return k > 0 ? k : 128;  // the documented default (ttk_ctx_set_knob rejects <= 0)
}

double *splitk_scratch(int64_t n) {  // partial-sum slabs of the current context (grown, never shrunk)
  ttk::Ctx &c = ttk::ctx();
  if (n > c.splitk_n) {
    if (c.splitk) {
      // earlier split-K launches may still read the old slab
      (void)(c.stream ? hipStreamSynchronize(c.stream) : hipDeviceSynchronize());
      (void)hipFree(c.splitk);
    }
    const int64_t want = n < (1 << 20) ? (1 << 20) : 2 * n;
    if (hipMalloc(reinterpret_cast<void **>(&c.splitk), want * sizeof(double)) != hipSuccess) {
      c.splitk = nullptr;
      c.splitk_n = 0;
      return nullptr;
    }
    c.splitk_n = want;
  }
  return c.splitk;
}

}  // namespace

// ttk_ctx_create: the slabs allocated with the context, so a launch-only entry point (which keeps
// the GIL, _lib.py) does not stall the process's other solve thread on a sync + hipMalloc later
int ttk::presize_splitk() { return splitk_scratch(1) ? TTK_OK : TTK_ERR_HIP; }

namespace {

// diagnostics: launch-shape histogram of the GEMM steps (ttk_gemm_hist)
bool g_hist_on = false;
std::map<std::array<int, 4>, std::pair<long long, double>> g_hist;
}  // namespace

extern "C" {

int ttk_gemm_set_splitk(int on) {
  int &k = ttk::ctx().knob[TTK_KNOB_SPLITK];
  const int old = k != 0 ? 1 : 0;
  k = on != 0;
  return old;
}

int ttk_gemm_hist(int on, const char *dump_path) {
  if (dump_path) {
    FILE *f = std::fopen(dump_path, "w");
    if (!f) return TTK_ERR_ARG;
    std::fprintf(f, "nb M N K launches flops\n");
    for (const auto &kv : g_hist)
      std::fprintf(f, "%d %d %d %d %lld %.6g\n", kv.first[0], kv.first[1], kv.first[2], kv.first[3],
                   kv.second.first, kv.second.second);
    std::fclose(f);
  }
  if (on < 0) g_hist.clear();
  g_hist_on = on > 0;
  return TTK_OK;
}

// K per split: splitk_mink(), 128 by default (round 3: the graphm_3 split-K shapes 6-16 % faster per call
// than at 256, and every whole-solve golden key follows a reference run under tests/parity_policy.py)
static int g_gemm64_min = getenv("TTK_GEMM64_MIN") ? atoi(getenv("TTK_GEMM64_MIN")) : 64;
static int g_gemm64_ks = getenv("TTK_GEMM64_KS") ? atoi(getenv("TTK_GEMM64_KS")) : 32;

int ttk_gemm_offs(void *stream, const double *A, const double *B, double *C, const int64_t *offs,
                  int nb, int M, int N, int K, double alpha, double beta) {
  if (nb <= 0 || M <= 0 || N <= 0) return TTK_OK;
  if (g_hist_on) {
    auto &e = g_hist[{nb, M, N, K}];
    e.first += 1;
    e.second += 2.0 * M * N * (double)K * nb;
  }
  if (K <= 0 || nb > 65535) {
    ttk::set_error("ttk_gemm_offs: bad shape nb=%d M=%d N=%d K=%d", nb, M, N, K);
    return TTK_ERR_ARG;
  }
  GemmArgs g{A, B, C, offs, nb, M, N, K, alpha, beta};
  dim3 grid((N + TN - 1) / TN, (M + TM - 1) / TM, nb);
  hipEvent_t e0, e1;
  int rc = contract_events(&e0, &e1);
  if (rc != TTK_OK) return rc;
  // split-K when the tile grid cannot fill the chip and K is long: each split runs >= splitk_mink() of K
  const int64_t tiles = (int64_t)grid.x * grid.y * nb;
  int nsplit = 1;
  if (splitk_on() && tiles < 256 && K >= 2 * splitk_mink()) {
    nsplit = (int)(K / splitk_mink());
    const int64_t cap = (512 + tiles - 1) / tiles;
    if (nsplit > cap) nsplit = (int)cap;
    if ((int64_t)nsplit * nb > 65535) nsplit = (int)(65535 / nb);
  }
  if (nsplit > 1) {
    const int kc = ((K + nsplit - 1) / nsplit + TK - 1) / TK * TK;
    nsplit = (K + kc - 1) / kc;
    double *part = splitk_scratch((int64_t)nsplit * nb * M * N);
    if (!part) {
      ttk::set_error("ttk_gemm_offs: split-K scratch allocation failed");
      return TTK_ERR_HIP;
    }
    dim3 gs(grid.x, grid.y, nb * nsplit);
    ttk::Ctx &cx = ttk::ctx();
    if (cx.knob[TTK_KNOB_SPLITK_FUSED] && tiles <= SPLITK_TILES_MAX) {
      if (!cx.splitk_cnt) {  // per-tile counters, zero between launches (each launch's last blocks reset them)
        TTK_HIP(hipMalloc(reinterpret_cast<void **>(&cx.splitk_cnt), SPLITK_TILES_MAX * sizeof(unsigned)));
        TTK_HIP(hipMemsetAsync(cx.splitk_cnt, 0, SPLITK_TILES_MAX * sizeof(unsigned), TTK_STREAM(stream)));
      }
      hipExtLaunchKernelGGL(gemm_offs_splitk_fused_kernel<64>, gs, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g,
                            nsplit, kc, part, cx.splitk_cnt);
    } else {
      hipExtLaunchKernelGGL(gemm_offs_splitk_kernel<64>, gs, dim3(256), 0, TTK_STREAM(stream), e0, nullptr, 0, g,
                            nsplit, kc, part);
      const int64_t tot = (int64_t)nb * M * N;
      hipExtLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                            TTK_STREAM(stream), nullptr, e1, 0, g, nsplit, part);
    }
  } else if (M >= g_gemm64_min && N >= g_gemm64_min && K >= 64 &&
             (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN) * nb >= 512) {
    dim3 g64((N + BN - 1) / BN, (M + BM - 1) / BM, nb);
    if (g_gemm64_ks == 32)
      hipExtLaunchKernelGGL(gemm_offs64_kernel<32>, g64, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g);
    else
      hipExtLaunchKernelGGL(gemm_offs64_kernel<16>, g64, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g);
  } else {
    switch (stage_k(K)) {
      case 16: hipExtLaunchKernelGGL(gemm_offs_kernel<16>, grid, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g); break;
      case 32: hipExtLaunchKernelGGL(gemm_offs_kernel<32>, grid, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g); break;
      default: hipExtLaunchKernelGGL(gemm_offs_kernel<64>, grid, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g);
    }
  }
  TTK_LAUNCH_CHECK();
  contract_count(2.0 * M * N * (double)K * nb);
  return TTK_OK;
}

}  // extern "C"

namespace ttk {

bool gemm_groupable(int nb, int M, int N, int K) {
  if (nb <= 0 || M <= 0 || N <= 0 || K <= 0 || nb > 65535) return false;
  const int64_t tiles = (int64_t)((N + TN - 1) / TN) * ((M + TM - 1) / TM) * nb;
  if (splitk_on() && tiles < 256 && K >= 2 * splitk_mink()) return false;  // split-K path
  if (M >= g_gemm64_min && N >= g_gemm64_min && K >= 64 &&
      (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN) * nb >= 512)
    return false;  // throughput variant: the problem fills the chip on its own
  return tiles <= 4096;
}

int gemm_group(hipStream_t st, const GemmProblem *p, int n) {
  for (int base = 0; base < n; base += GROUP_MAX) {
    GemmGroup G;
    G.n = n - base < GROUP_MAX ? n - base : GROUP_MAX;
    G.tile0[0] = 0;
    double flops = 0.0;
    int kmax = 0;
    for (int i = 0; i < G.n; ++i) {
      const GemmProblem &q = p[base + i];
      kmax = q.K > kmax ? q.K : kmax;
      G.p[i] = GemmArgs{q.A, q.B, q.C, q.offs, q.nb, q.M, q.N, q.K, q.alpha, q.beta};
      G.tile0[i + 1] = G.tile0[i] + ((q.N + TN - 1) / TN) * ((q.M + TM - 1) / TM) * q.nb;
      flops += 2.0 * q.M * q.N * (double)q.K * q.nb;
    }
    hipEvent_t e0, e1;
    int rc = contract_events(&e0, &e1);
    if (rc != TTK_OK) return rc;
    switch (stage_k(kmax)) {
      case 16: hipExtLaunchKernelGGL(gemm_offs_group_kernel<16>, dim3(G.tile0[G.n]), dim3(256), 0, st, e0, e1, 0, G); break;
      case 32: hipExtLaunchKernelGGL(gemm_offs_group_kernel<32>, dim3(G.tile0[G.n]), dim3(256), 0, st, e0, e1, 0, G); break;
      default: hipExtLaunchKernelGGL(gemm_offs_group_kernel<64>, dim3(G.tile0[G.n]), dim3(256), 0, st, e0, e1, 0, G);
    }
    TTK_LAUNCH_CHECK();
    contract_count(flops);
  }
  return TTK_OK;
}

}  // namespace ttk

extern "C" {

int ttk_gemm_offs_grouped(void *stream, const double *const *Aptr, const double *const *Bptr,
                          double *const *Cptr, const int64_t *offs, int ngroups, int nb, int M,
                          int N, int K, double alpha, double beta) {
  if (ngroups <= 0 || nb <= 0 || M <= 0 || N <= 0) return TTK_OK;
  if (K <= 0 || (int64_t)nb * ngroups > 65535) {
    ttk::set_error("ttk_gemm_offs_grouped: bad shape");
    return TTK_ERR_ARG;
  }
  GemmArgs g{nullptr, nullptr, nullptr, offs, nb, M, N, K, alpha, beta};
  GroupPtrs p{Aptr, Bptr, Cptr};
  dim3 grid((N + TN - 1) / TN, (M + TM - 1) / TM, nb * ngroups);
  hipEvent_t e0, e1;
  int rc = contract_events(&e0, &e1);
  if (rc != TTK_OK) return rc;
  switch (stage_k(K)) {
    case 16: hipExtLaunchKernelGGL(gemm_offs_grouped_kernel<16>, grid, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g, p); break;
    case 32: hipExtLaunchKernelGGL(gemm_offs_grouped_kernel<32>, grid, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g, p); break;
    default: hipExtLaunchKernelGGL(gemm_offs_grouped_kernel<64>, grid, dim3(256), 0, TTK_STREAM(stream), e0, e1, 0, g, p);
  }
  TTK_LAUNCH_CHECK();
  contract_count(2.0 * M * N * (double)K * nb * ngroups);
  return TTK_OK;
}

int ttk_copy_nd(void *stream, const double *src, double *dst, int ndim, const int64_t *shape,
                const int64_t *sstride, const int64_t *dstride, double alpha, double beta) {
  if (int rc = ttk::batch_barrier(stream)) return rc;
  ttk::NdDesc d;
  int st = make_nd(d, ndim, shape, sstride, dstride, nullptr);
  if (st) return st;
  if (d.total == 0) return TTK_OK;
  hipLaunchKernelGGL(copy_nd_kernel, dim3(grid_for(d.total, 256)), dim3(256), 0, TTK_STREAM(stream), src,
                     dst, d, alpha, beta);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_mul_nd(void *stream, const double *src, const double *src2, double *dst, int ndim,
               const int64_t *shape, const int64_t *sstride, const int64_t *s2stride,
               const int64_t *dstride, double alpha, double beta) {
  if (int rc = ttk::batch_barrier(stream)) return rc;
  ttk::NdDesc d;
  int st = make_nd(d, ndim, shape, sstride, s2stride, dstride);
  if (st) return st;
  if (d.total == 0) return TTK_OK;
  hipLaunchKernelGGL(mul_nd_kernel, dim3(grid_for(d.total, 256)), dim3(256), 0, TTK_STREAM(stream), src,
                     src2, dst, d, alpha, beta);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_axpby_nd(void *stream, const double *src, const double *src2, double *dst, int ndim, const int64_t *shape,
                 const int64_t *sstride, const int64_t *s2stride, const int64_t *dstride, double alpha, double beta,
                 double gamma) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  ttk::NdDesc d;
  int st = make_nd(d, ndim, shape, sstride, s2stride, dstride);
  if (st) return st;
  if (d.total == 0) return TTK_OK;
  hipLaunchKernelGGL(axpby_nd_kernel, dim3(grid_for(d.total, 256)), dim3(256), 0, TTK_STREAM(stream), src, src2, dst,
                     d, alpha, beta, gamma);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_tt_join(void *stream, const double *a, const double *b, double *out, int ra, int Ra, int rb, int Rb,
                int64_t mid, int mode) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (mode < 0 || mode > 2 || (mode == 1 && ra != rb) || (mode == 2 && Ra != Rb)) {
    ttk::set_error("ttk_tt_join: bad mode %d / shapes", mode);
    return TTK_ERR_ARG;
  }
  const int64_t total = (int64_t)(mode == 1 ? ra : ra + rb) * mid * (mode == 2 ? Ra : Ra + Rb);
  if (total == 0) return TTK_OK;
  hipLaunchKernelGGL(tt_join_kernel, dim3(grid_for(total, 256)), dim3(256), 0, TTK_STREAM(stream), a, b, out, ra, Ra,
                     rb, Rb, mid, mode);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_scale_axis(void *stream, const double *src, double *dst, int ndim, const int64_t *shape,
                   const int64_t *sstride, const int64_t *dstride, int axis, const double *scales) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  ttk::NdDesc d;
  int st = make_nd(d, ndim, shape, sstride, dstride, nullptr);
  if (st) return st;
  if (axis < 0 || axis >= ndim || shape[axis] > 16) {
    ttk::set_error("ttk_scale_axis: axis %d (extent %lld) out of range (max extent 16)", axis,
                   axis >= 0 && axis < ndim ? (long long)shape[axis] : -1LL);
    return TTK_ERR_ARG;
  }
  if (d.total == 0) return TTK_OK;
  AxisScales sc;
  for (int i = 0; i < 16; ++i) sc.v[i] = i < shape[axis] ? scales[i] : 0.0;
  hipLaunchKernelGGL(scale_axis_kernel, dim3(grid_for(d.total, 256)), dim3(256), 0, TTK_STREAM(stream), src, dst,
                     d, axis, sc);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_scale_axis_ss(void *stream, const double *src, double *dst, int ndim, const int64_t *shape,
                      const int64_t *sstride, const int64_t *dstride, int axis, const double *ss, int invert) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  ttk::NdDesc d;
  int st = make_nd(d, ndim, shape, sstride, dstride, nullptr);
  if (st) return st;
  if (axis < 0 || axis >= ndim) {
    ttk::set_error("ttk_scale_axis_ss: axis %d out of range", axis);
    return TTK_ERR_ARG;
  }
  if (d.total == 0) return TTK_OK;
  hipLaunchKernelGGL(scale_axis_ss_kernel, dim3(grid_for(d.total, 256)), dim3(256), 0, TTK_STREAM(stream), src, dst,
                     d, axis, ss, invert);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_recip(void *stream, const double *src, double *dst, int64_t n) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (n <= 0) return TTK_OK;
  hipLaunchKernelGGL(recip_kernel, dim3(grid_for(n, 256)), dim3(256), 0, TTK_STREAM(stream), src, dst, n);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_copy_many(void *stream, int n, const double *const *src, double *const *dst, const int64_t *count) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  for (int i0 = 0; i0 < n; i0 += CopyMany::MAXN) {
    CopyMany m{};
    m.n = n - i0 < CopyMany::MAXN ? n - i0 : CopyMany::MAXN;
    m.off[0] = 0;
    for (int j = 0; j < m.n; ++j) {
      m.src[j] = src[i0 + j];
      m.dst[j] = dst[i0 + j];
      m.off[j + 1] = m.off[j] + (count[i0 + j] > 0 ? count[i0 + j] : 0);
    }
    if (m.off[m.n] == 0) continue;
    hipLaunchKernelGGL(copy_many_kernel, dim3(grid_for(m.off[m.n], 256)), dim3(256), 0, TTK_STREAM(stream), m);
    TTK_LAUNCH_CHECK();
  }
  return TTK_OK;
}

int ttk_fill(void *stream, double *dst, int64_t n, double value) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (n <= 0) return TTK_OK;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n, 256)), dim3(256), 0, TTK_STREAM(stream), dst, n, value);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_add_diag(void *stream, double *A, int n, int lda, double value) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (n <= 0) return TTK_OK;
  hipLaunchKernelGGL(add_diag_kernel, dim3(grid_for(n, 256)), dim3(256), 0, TTK_STREAM(stream), A, n, lda, value);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_dot_nd_sync(void *stream, const double *x, const double *y, int ndim, const int64_t *shape,
                    const int64_t *xstride, const int64_t *ystride, double *result) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  ttk::NdDesc d;
  int st = make_nd(d, ndim, shape, xstride, ystride, nullptr);
  if (st) return st;
  if (!ttk::ctx().dev_scalar) TTK_HIP(hipMalloc(reinterpret_cast<void **>(&ttk::ctx().dev_scalar), 64 * sizeof(double)));
  if (d.total == 0) {
    *result = 0.0;
    return TTK_OK;
  }
  static const int mapped = getenv("TTK_MAPPED_READS") ? atoi(getenv("TTK_MAPPED_READS")) : 1;
  double *dev = nullptr;
  double *h = mapped ? ttk::mapped_stage(1, &dev) : nullptr;  // the reduction writes to host-coherent memory
  hipLaunchKernelGGL(dot_nd_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), x, y, d, h ? dev : ttk::ctx().dev_scalar);
  TTK_LAUNCH_CHECK();
  if (!h) return ttk_read_sync(stream, ttk::ctx().dev_scalar, result, 1);
  ttk::note_sync();
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  *result = h[0];
  return TTK_OK;
}

int ttk_dot_nd_dev(void *stream, const double *x, const double *y, int ndim, const int64_t *shape,
                   const int64_t *xstride, const int64_t *ystride, double *out) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  ttk::NdDesc d;
  int st = make_nd(d, ndim, shape, xstride, ystride, nullptr);
  if (st) return st;
  if (d.total == 0) {
    hipLaunchKernelGGL(fill_kernel, dim3(1), dim3(64), 0, TTK_STREAM(stream), out, (int64_t)1, 0.0);
  } else {
    hipLaunchKernelGGL(dot_nd_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), x, y, d, out);
  }
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_normalize(void *stream, const double *x, double *out, int ndim, const int64_t *shape,
                  const int64_t *xstride) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  ttk::NdDesc d;
  int64_t ost[ttk::MAXD];
  if (ndim > ttk::MAXD || ndim < 0) {
    ttk::set_error("ttk_normalize: ndim %d", ndim);
    return TTK_ERR_ARG;
  }
  int64_t acc = 1;
  for (int i = ndim - 1; i >= 0; --i) {
    ost[i] = acc;
    acc *= shape[i];
  }
  int st = make_nd(d, ndim, shape, xstride, xstride, ost);
  if (st) return st;
  if (d.total == 0) return TTK_OK;
  hipLaunchKernelGGL(normalize_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), x, d, out);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_rayleigh_tail_sync(void *stream, const double *v, double *Mv, int64_t n, double *ev_out, double *res2_out) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  double *dev = nullptr;
  double *h = ttk::mapped_stage(2, &dev);
  if (!h) {
    ttk::set_error("ttk_rayleigh_tail_sync: mapped allocation failed");
    return TTK_ERR_HIP;
  }
  hipLaunchKernelGGL(rayleigh_tail_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), v, Mv, n, dev, 1.0);
  TTK_LAUNCH_CHECK();
  ttk::note_sync();
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  *ev_out = h[0];
  *res2_out = h[1];
  return TTK_OK;
}

// the same tail with (ev, ||Mv - ev v||^2) left in device memory (read later, batched with others)
int ttk_rayleigh_tail_dev(void *stream, const double *v, double *Mv, int64_t n, double *out2) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  hipLaunchKernelGGL(rayleigh_tail_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), v, Mv, n, out2, 1.0);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_sumsq_batched(void *stream, const double *x, int64_t n, int nb, int64_t bstride, double *out) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (nb <= 0) return TTK_OK;
  hipLaunchKernelGGL(sumsq_batched_kernel, dim3(nb), dim3(256), 0, TTK_STREAM(stream), x, n, bstride, out);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_sumsq_batched_strided(void *stream, const double *x, int64_t n, int nb, int64_t bstride, int64_t inner,
                              int64_t ostride, double *out) {
  if (int brc = ttk::batch_barrier(stream)) return brc;  // an open einsum batch may feed this call
  if (nb <= 0) return TTK_OK;
  if (inner <= 0) {
    ttk::set_error("ttk_sumsq_batched_strided: inner %lld", (long long)inner);
    return TTK_ERR_ARG;
  }
  hipLaunchKernelGGL(sumsq_batched2_kernel, dim3(nb), dim3(256), 0, TTK_STREAM(stream), x, n, bstride, inner, ostride,
                     out);
  TTK_LAUNCH_CHECK();
  return TTK_OK;
}

int ttk_rank_scan_sync(void *stream, double *res, const double *negs, int64_t n, int nq, double *host_out) {
  if (nq <= 0) return TTK_OK;
  if (int rc = ttk::batch_barrier(stream)) return rc;
  double *dev = nullptr;
  double *h = ttk::mapped_stage((size_t)nq, &dev);
  if (!h) {
    ttk::set_error("ttk_rank_scan_sync: mapped buffer allocation failed");
    return TTK_ERR_HIP;
  }
  hipLaunchKernelGGL(rank_scan_kernel, dim3(1), dim3(1024), 0, TTK_STREAM(stream), res, negs, n, nq, dev);
  TTK_LAUNCH_CHECK();
  ttk::note_sync();
  TTK_HIP(hipStreamSynchronize(TTK_STREAM(stream)));
  std::memcpy(host_out, h, (size_t)nq * sizeof(double));
  return TTK_OK;
}

int ttk_contract_timing(int on) {
  const int old = g_cs.timing;
  if (!on && g_cs.timing) {
    int rc = harvest_events();
    if (rc != TTK_OK) return rc;
  }
  g_cs.timing = on != 0;
  return old;
}

int ttk_contract_stats(double *out, int reset) {
  int rc = harvest_events();
  if (rc != TTK_OK) return rc;
  out[0] = g_cs.flops;
  out[1] = (double)g_cs.launches;
  out[2] = g_cs.timed_flops;
  out[3] = (double)g_cs.timed_launches;
  out[4] = g_cs.timed_ms;
  if (reset) {
    g_cs.flops = g_cs.timed_flops = g_cs.timed_ms = 0.0;
    g_cs.launches = g_cs.timed_launches = 0;
  }
  return TTK_OK;
}

}  // extern "C"
