/*
 * ttk.h -- C ABI of the MI355X (gfx950) TT-IPM hot-path library `libttk.so`.
 *
 * The reference has no C ABI: its native boundary is the Cython module surface
 * (`cy_src/tt_ops_cy.pyx`, `cy_src/lgmres_cy.pyx`) plus LAPACK/PETSc reached through SciPy and
 * petsc4py.  Every entry point below replaces one of those native calls; the
 * reference interface each one stands in for is cited next to it.  The Python host layer
 * (`ttipm_amd`) re-exposes them under the reference's names (tt_rank_reduce, MatVecWrapper, ...).
 *
 * Conventions
 *   - all tensors are fp64, device-resident, caller-owned (the library never frees caller memory);
 *   - strided operands are described by int64 offset tables that live in device memory
 *     (built once per (equation, shapes) plan on the host and cached, like the reference's
 *     LRU-cached opt_einsum expressions, `src/tt_ops.py:22-28`);
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *   - every function returns an int status (TTK_OK = 0); no C++ exception crosses the ABI;
 *     `ttk_last_error()` returns a thread-local message for the last failure;
 *   - functions whose name ends in `_sync` block on `stream` and return host scalars that drive
 *     host-side decisions (rank truncation, convergence tests);
 *   - threading: one host thread per context (ttk_ctx below); all scratch, staging and handle
 *     state is per context, the einsum plan cache is shared and lock-protected.  The roofline
 *     statistics (ttk_contract_stats / _timing) are process-wide.
 */
#ifndef TTK_H
#define TTK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ttk_status {
  TTK_OK = 0,
  TTK_ERR_ARG = 1,          /* invalid argument / shape */
  TTK_ERR_HIP = 2,          /* HIP runtime error */
  TTK_ERR_NOT_PD = 3,       /* Cholesky: matrix not positive definite (scipy LinAlgError) */
  TTK_ERR_SINGULAR = 4,     /* LU / triangular: exact zero pivot (scipy LinAlgError) */
  TTK_ERR_NOT_CONVERGED = 5, /* iterative kernel hit its sweep cap */
  TTK_ILL_CONDITIONED = 6    /* LU: rcond < eps/2 (scipy's LinAlgWarning, raised as an error) */
};

/* ---------------------------------------------------------------------------------------
 * Contexts.  A context owns every piece of mutable library state between calls -- einsum
 * intermediates and batch recorder, split-K slabs, LGMRES partials, Schur operator handles,
 * factorisation status words, the pinned upload ring and the host-coherent read buffer -- and
 * the HIP stream its work goes to.  Entry points taking a ttk_ctx run on that context; the older
 * entry points (taking a stream) run on the calling thread's bound context (ttk_ctx_bind), or on
 * the process default context when none is bound.  Two contexts driven by two host threads on two
 * streams of one GPU share only the (lock-protected, immutable-once-built) einsum plan cache, so
 * several seeds can be solved concurrently on one device.  Schur handles are per context.
 * ------------------------------------------------------------------------------------- */
typedef struct ttk_ctx_s *ttk_ctx;
int ttk_ctx_create(void *stream, ttk_ctx *out);
int ttk_ctx_destroy(ttk_ctx ctx);      /* synchronises the context's stream, frees its buffers */
int ttk_ctx_bind(ttk_ctx ctx);         /* make ctx current for the calling thread (NULL: default) */
void *ttk_ctx_stream(ttk_ctx ctx);

/* Numerics knobs, per context.  Each changes which kernel variant (and so which summation order)
 * a call uses; they live in the context so that flipping one for one context never changes the
 * results of another.  ctx NULL: the calling thread's current context (bound or default).
 *   FUSED_APPLY     1: local applies opted in by the caller run on the one-launch fused kernel
 *                      (default from env TTK_FUSED_APPLY, else 1)
 *   FUSED_MFMA      1: fused applies beyond the VALU kernel's FLOP range run the MFMA stages
 *                      (default from env TTK_FUSED_MFMA, else 1); 0: the pairwise plan
 *   SPLITK          1: deterministic split-K for GEMM steps whose tile grid cannot fill the chip
 *                      (default from env TTK_SPLITK, else 1)
 *   SPLITK_MINK     K per split, > 0 (default from env TTK_SPLITK_MINK, else 128; ttk_ctx_set_knob
 *                   rejects values <= 0 with TTK_ERR_ARG)
 *   LGMRES_MW_MIN   (it+1)*n at or above which the LGMRES Arnoldi / build / augmentation steps
 *                   run as multi-workgroup kernels (default from env TTK_LGMRES_MW_MIN, else
 *                   16384; 0 everywhere, INT_MAX never)
 *   MFMA_CSPLIT     1: wide MFMA-stage apply rows spread their stage-3 output tiles over several
 *                   workgroups per row (bit-identical; default from env TTK_MFMA_CSPLIT, else 1)
 *   APPLY_DUAL      1: a Schur-handle task's two VALU terms run side by side, one half of a
 *                   512-thread workgroup each (bit-identical; read at ttk_schur_build; default from
 *                   env TTK_APPLY_DUAL, else 1)
 *   RCOND_EXACT     1: ttk_lu_sync / ttk_dense_schur_solve always run dgecon's estimator, so
 *                   rcond_out is dgecon's value; 0 (default from env TTK_RCOND_EXACT, else 0): a
 *                   certified lower bound may be returned instead when it settles the rcond < eps
 *                   test (the status is identical either way; see ttk_lu_sync)
 *   SCHUR_ONE       1: a fused Schur matvec (ttk_schur_apply) is ONE launch: the o1 = B21 x - B22 w
 *                   rows compute B21 x while the w = inv_I o B01^T y rows run, then take w over an
 *                   in-launch hand-off; 0: two launches (bit-identical either way; default from env
 *                   TTK_SCHUR_ONE, else 1)
 *   ARNOLDI_ONE     1: a multi-workgroup LGMRES Arnoldi step (partial dots, basis update, norm +
 *                   Hessenberg/Givens) is ONE launch over in-launch hand-offs; 0: three launches
 *                   (bit-identical either way; default from env TTK_ARNOLDI_ONE, else 0 since round 6:
 *                   the three launches measured 7.5 % faster per graphm_3 r=2 solve, maxcut within
 *                   noise -- profiles/r06_ab_knobs_graphm3.txt)
 *   SCHUR_PREP      1: ttk_schur_build copies every term's A (and VALU rows' Q) once into the
 *                   layout the apply rows stage in LDS, so a matvec stages them with contiguous
 *                   copies instead of strided gathers (bit-identical; read at build; default
 *                   from env TTK_SCHUR_PREP, else 1)
 * TTK_KNOB_SPLITK_FUSED  1: a split-K GEMM is ONE launch -- the split blocks of a tile store their
 *                   partial tiles write-through and count their arrival; the last one to arrive sums
 *                   the partials in split order and writes C (the separate reduce launch's
 *                   arithmetic, bit-identical); 0: split kernel + reduce kernel (default from env
 *                   TTK_SPLITK_FUSED, else 1)
 * TTK_KNOB_TRI_HOIST  1: each step of the multi-workgroup Householder tridiagonalisation of
 *                   ttk_syev_extreme (128 < n <= 512) issues every global load of the step before
 *                   its first use -- one L2 round trip per step instead of three; 0: the loads
 *                   where they are used (same arithmetic in the same order: bit-identical; default
 *                   from env TTK_TRI_HOIST, else 1)
 * TTK_KNOB_TRI_ONE    largest n (<= 513) whose Householder tridiagonalisation in ttk_syev_extreme runs
 *                   as ONE one-workgroup launch (tri_wg_kernel: the per-step launches' arithmetic,
 *                   bit-identical) instead of one launch per Householder step; 0: never (default from
 *                   env TTK_TRI_ONE, else 0: measured slower per call from n = 144 on -- one CU's L2
 *                   bandwidth and serial latency against 64 workgroups per step)
 * TTK_KNOB_SVD_SWEEP_ONE  1: the multi-workgroup one-sided Jacobi of ttk_svd (min(m,n) > 96) runs
 *                   ONE launch per sweep -- the pair waves stay resident for every round and hand
 *                   columns to the next round through per-column counters (in-launch hand-offs);
 *                   0: one launch per round-robin round (the same rotations in the same order:
 *                   bit-identical; default from env TTK_SVD_SWEEP_ONE, else 0: measured 1.3-1.8x
 *                   slower per SVD -- a column hand-off through memory costs more than the launch
 *                   boundary it replaces, profiles/r06_persist.txt)
 * TTK_KNOB_TRI_PERSIST  1: the per-step launches of TTK_KNOB_TRI_HOIST (128 < n <= 512) become ONE
 *                   launch whose resident workgroups run every step, handing each step's words to the
 *                   next through the context's arrival counter (in-launch hand-offs); 0: one launch per
 *                   step (the same step code: bit-identical; default from env TTK_TRI_PERSIST, else 0:
 *                   measured 1.3-2.4x slower per eigenpair, profiles/r06_persist.txt)
 * TTK_KNOB_SYEV_WAVES8  1: the small extreme-eigenpair kernel (n < 64) runs 8 waves -- the same symv
 *                   (2 lanes per row), the rank-2 row updates spread over 7 waves instead of 3; 0: 4
 *                   waves (bit-identical; default from env TTK_SYEV_WAVES8, else 1: 4-9 % faster per call
 *                   from n = 32 on, equal below, profiles/r06_syev_small.txt)
 * TTK_KNOB_BT_STAGE  1: the back-transform of the multi-launch extreme eigenpair (128 < n <= 513) reads
 *                   its reflectors from LDS blocks that the finish kernel's idle waves stage while wave
 *                   0 applies the previous block; 0: each reflector loaded from global memory one ahead
 *                   (bit-identical; default from env TTK_BT_STAGE, else 1: 3-5 % faster per eigenpair,
 *                   profiles/r06_bt_stage.txt)
 * ttk_ctx_set_knob stores value and returns the previous one in *old (may be NULL). */
enum ttk_knob {
  TTK_KNOB_FUSED_APPLY = 0,
  TTK_KNOB_FUSED_MFMA = 1,
  TTK_KNOB_SPLITK = 2,
  TTK_KNOB_SPLITK_MINK = 3,
  TTK_KNOB_LGMRES_MW_MIN = 4,
  TTK_KNOB_MFMA_CSPLIT = 5,
  TTK_KNOB_APPLY_DUAL = 6,
  TTK_KNOB_RCOND_EXACT = 7,
  TTK_KNOB_SCHUR_ONE = 8,
  TTK_KNOB_ARNOLDI_ONE = 9,
  TTK_KNOB_SCHUR_PREP = 10,
  TTK_KNOB_SPLITK_FUSED = 11,
  TTK_KNOB_TRI_HOIST = 12,
  TTK_KNOB_TRI_ONE = 13,
  TTK_KNOB_SVD_SWEEP_ONE = 14,
  TTK_KNOB_TRI_PERSIST = 15,
  TTK_KNOB_SYEV_WAVES8 = 16,
  TTK_KNOB_BT_STAGE = 17,
  TTK_KNOB_COUNT = 18
};
int ttk_ctx_set_knob(ttk_ctx ctx, int knob, int value, int *old);
int ttk_ctx_get_knob(ttk_ctx ctx, int knob, int *value);

const char *ttk_last_error(void);
int ttk_version(void);
/* number of kernel launches issued since load (profiling / launch-count tests) */
long long ttk_launch_count(void);
/* host waits on a stream so far (every device scalar the host branches on costs one) */
long long ttk_sync_count(void);

/* ---------------------------------------------------------------------------------------
 * Contractions.  One pairwise step of a planned einsum:
 *   C[b,m,n] = alpha * sum_k A[b,m,k] * B[b,k,n] + beta * C[b,m,n]
 * with A[b,m,k] = A[a_b[b] + a_m[m] + a_k[k]] etc.  `offs` (device, int64) holds the nine
 * offset tables back to back: a_b(nb) a_m(M) a_k(K) b_b(nb) b_k(K) b_n(N) c_b(nb) c_m(M) c_n(N).
 * fp64 MFMA (v_mfma_f64_16x16x4_f64), 32x32 output tile per 256-thread workgroup, K staged
 * through LDS.  Replaces every `cached_einsum` / `np.tensordot` step on the path
 * (`src/tt_ops.py:26-28`, `src/tt_als.py:190-265`, `cy_src/tt_ops_cy.pyx:399,413,441,458`)
 * and the dgemm chain of `MatVecWrapper` (`cy_src/lgmres_cy.pyx:36-49,126-153`).
 * ------------------------------------------------------------------------------------- */
int ttk_gemm_offs(void *stream, const double *A, const double *B, double *C, const int64_t *offs,
                  int nb, int M, int N, int K, double alpha, double beta);

/* Grouped variant: `ngroups` independent GEMMs of identical (nb,M,N,K) in one launch; operand
 * base pointers are device arrays of pointers (group g uses Aptr[g], Bptr[g], Cptr[g]). */
int ttk_gemm_offs_grouped(void *stream, const double *const *Aptr, const double *const *Bptr,
                          double *const *Cptr, const int64_t *offs, int ngroups, int nb, int M,
                          int N, int K, double alpha, double beta);
/* Native einsum engine (replaces `cached_einsum`, src/tt_ops.py:22-28, and the tensordot chains
 * of cy_src/tt_ops_cy.pyx): out = alpha * einsum(eq, ops) + beta * out on device fp64 data.
 * desc = [nops | (allow_fused << 8), {ptr, ndim, shape[ndim], stride[ndim]} x nops, has_out_strides,
 * (ndim, out_stride[ndim])], strides in elements (views need not be contiguous).  Plans (greedy
 * pairwise order + offset tables) are cached per (eq, shapes, strides); each pairwise step is one
 * ttk_gemm_offs launch. */
int ttk_einsum(void *stream, const char *eq, const int64_t *desc, double *out, double alpha, double beta);

/* Einsum batches: between begin and end, ttk_einsum records its steps (same plans, same fused-apply
 * decisions, private intermediates) instead of launching them; end (or flush) launches them level
 * by level -- a level is a set of steps without read/write conflicts -- as one grouped MFMA GEMM
 * launch plus one grouped fused-apply launch per level.  Bit-identical to the unbatched calls.
 * Used for one AMEn core step's environment updates (`src/tt_als.py:372-387,499-514`), the
 * block local products and the rank loop's candidate products (`src/tt_als.py:334-346`).
 * Every other entry point that takes a stream (element-wise, reductions, reads, factorisations,
 * LGMRES steps) flushes the pending steps first, so stream order holds for C callers that read
 * an einsum output while a batch is open.  Nesting is counted; every end (nested ones included)
 * launches what is pending.  stats: [flushes, recorded steps, launches]. */
/* Local applies beyond the VALU fused kernel's FLOP range (graphm-sized blocks) run the same three
 * stages on fp64 MFMA in one launch (one workgroup per output row) when they fit LDS; off: the
 * pairwise plan.  Returns the previous setting (default on; env TTK_FUSED_MFMA=0 turns it off).
 * Shorthand for ttk_ctx_set_knob(NULL, TTK_KNOB_FUSED_MFMA, ...): the current context only. */
int ttk_fused_set_mfma(int on);
/* diagnostics: per-phase wall-clock sums (100 MHz ticks) of the MFMA rows in a -DTTK_MFMA_PROFILE
 * build: [staging, stage 1, stage 2, stage 3, epilogue, -, -, rows]; zeros otherwise */
int ttk_mfma_profile(unsigned long long *out8, int reset);
/* number of in-launch hand-off waits (one-launch Schur matvec, TTK_KNOB_SCHUR_ONE) that gave up
 * after their spin bound instead of hanging -- 0 unless something is broken; reset: zero it */
int ttk_dep_timeouts(unsigned *out, int reset);

int ttk_einsum_batch_begin(void *stream);
int ttk_einsum_batch_flush(void *stream);
int ttk_einsum_batch_end(void *stream);
int ttk_einsum_batch_stats(long long *out3);

/* Environment (interface) updates of one AMEn / ALS core step, every block in one call
 * (`compute_phi_fwd_A` / `compute_phi_bck_A`, `src/tt_als.py:252-257`, applied to all blocks of the
 * step, `src/tt_als.py:372-387,499-514`):
 *   forward   out[L,S,R] = sum phi[l,s,r] x[l,M,L] A[s,M,N,S] y[r,N,R]
 *   backward  out[l,s,r] = sum phi[L,S,R] x[l,M,L] A[s,M,N,S] y[r,N,R]
 * phi, x, y, out contiguous; A through a_strides (a transposed operator block is a stride swap).
 * Recorded as one einsum batch on the context's stream (grouped launches), so the results equal
 * nblocks separate relabelled local applies bit for bit. */
typedef struct {
  const double *phi;
  const double *x;
  const double *A;
  const double *y;
  double *out;
  int64_t phi_shape[3], x_shape[3], A_shape[4], y_shape[3];
  int64_t a_strides[4];
} ttk_env_block;
int ttk_env_update(ttk_ctx ctx, int backward, int nblocks, const ttk_env_block *blocks);

/* AMEn rank loop (`src/tt_als.py:334-346`, `:462-472`): res (n contiguous doubles) is updated
 * res <- res - negs[q] for q = 0..nq-1 in order and <res, res> after each update is returned in
 * host_out[q]; one launch and one host read for every candidate rank, with the same operations and
 * reduction order as nq separate copy_nd + dot_nd_sync calls. */
int ttk_rank_scan_sync(void *stream, double *res, const double *negs, int64_t n, int nq, double *host_out);
/* calls that opt in (desc flag) route 'lsr,smnS,LSR,rnR->lmL' / 'lsr,smnS,LSR,lmL->rnR' (the local
 * operator, src/tt_als.py:190-200, cy_src/lgmres_cy.pyx:126-153) to a one-launch fused kernel when
 * its intermediates fit LDS; this switch disables it for the current context (TTK_KNOB_FUSED_APPLY).
 * Returns the previous setting. */
int ttk_einsum_set_fused(int on);
/* out[3] = {plan hits, plan misses, cached plans} */
int ttk_einsum_stats(long long *out);
/* contraction-kernel accounting for the roofline report: on != 0 brackets every ttk_gemm_offs*
 * launch with two HIP events on its stream (returns the previous setting) */
int ttk_contract_timing(int on);
/* out[5] = {algorithmic FLOPs (2*M*N*K*batch per GEMM step), launches, timed FLOPs,
 * timed launches, summed kernel ms of the timed launches}; synchronises pending events */
int ttk_contract_stats(double *out, int reset);

/* split-K for GEMM steps whose tile grid cannot fill the chip (< 256 tiles) and K >= 2 x SPLITK_MINK: the K
 * range is split over workgroups into partial slabs summed in a fixed order by a second kernel.
 * on = 0 disables it for the current context (TTK_KNOB_SPLITK).  Returns the previous setting. */
int ttk_gemm_set_splitk(int on);
/* diagnostics: on > 0 records a (nb,M,N,K) histogram of ttk_gemm_offs launches, on < 0 clears it;
 * dump_path != NULL writes "nb M N K launches flops" lines */
int ttk_gemm_hist(int on, const char *dump_path);
/* diagnostics: on > 0 records a (kind, a, b, path) histogram of the dense factorisations (svd: a x b,
 * qr: a x b, syev_extreme: n and which, lu / cholesky: n), each recorded call bracketed by two stream
 * synchronisations and timed on the host; on < 0 clears it; dump_path != NULL writes
 * "kind a b path calls total_us" lines.  Never on in a timed run. */
int ttk_linalg_hist(int on, const char *dump_path);

/* ---------------------------------------------------------------------------------------
 * Strided element-wise kernels (up to 6-D).  `shape`, `sstride`, `dstride` are host arrays.
 * copy:  dst = alpha * src + beta * dst     (tt_add block-diagonal assembly
 *        `cy_src/tt_ops_cy.pyx:228-258`, transposes/permute copies, tt_scale `:94-114`)
 * mul:   dst = alpha * src * src2 + beta*dst (inv_I o v, `cy_src/lgmres_cy.pyx:107-120`)
 * recip: dst = 1 / src                        (`np.divide(1, ...)`, `src/tt_ipm.py:191`)
 * ------------------------------------------------------------------------------------- */
int ttk_copy_nd(void *stream, const double *src, double *dst, int ndim, const int64_t *shape,
                const int64_t *sstride, const int64_t *dstride, double alpha, double beta);
int ttk_mul_nd(void *stream, const double *src, const double *src2, double *dst, int ndim,
               const int64_t *shape, const int64_t *sstride, const int64_t *s2stride,
               const int64_t *dstride, double alpha, double beta);
int ttk_recip(void *stream, const double *src, double *dst, int64_t n);
/* n contiguous copies dst[i][0:count[i]] = src[i][0:count[i]] in one launch (the core copies of a
 * TT before an in-place rounding or scaling: the reference rebinds list entries and never writes
 * the caller's cores, cy_src/tt_ops_cy.pyx:179-226); src/dst/count are host arrays of n entries. */
int ttk_copy_many(void *stream, int n, const double *const *src, double *const *dst, const int64_t *count);
/* tt_add core assembly (`_block_diag_tensor` / concatenation, cy_src/tt_ops_cy.pyx:228-258) in one
 * launch from contiguous cores a (ra, mid, Ra), b (rb, mid, Rb): mode 0 block diagonal, 1 concat
 * along the last axis (ra == rb), 2 along the first axis (Ra == Rb); out contiguous. */
int ttk_tt_join(void *stream, const double *a, const double *b, double *out, int ra, int Ra, int rb,
                int Rb, int64_t mid, int mode);
/* dst = alpha * src + beta * (gamma * src2) in one launch, rounding like the two-step scaled +
 * copy it replaces (eigen-ALS M = A / step + D and (M + M^T) / 2, src/tt_als.py:957-996). */
int ttk_axpby_nd(void *stream, const double *src, const double *src2, double *dst, int ndim,
                 const int64_t *shape, const int64_t *sstride, const int64_t *s2stride,
                 const int64_t *dstride, double alpha, double beta, double gamma);
/* out (contiguous) = x / ||x||_2 on the device, no host round trip; bit-identical to
 * ttk_dot_nd_sync + host sqrt/reciprocal + ttk_copy_nd (`v / np.linalg.norm(v)` of the eigen-ALS,
 * src/tt_als.py:1002,1035).  A zero vector gives inf/nan instead of the host's ZeroDivisionError. */
int ttk_normalize(void *stream, const double *x, double *out, int ndim, const int64_t *shape,
                  const int64_t *xstride);
/* dst = src * f(ss[i_axis]) with f = max(sqrt(ss), 1e-10) (invert = 0) or its reciprocal: the
 * per-block scaling of the sweep from the device block sums of squares (no host read). */
int ttk_scale_axis_ss(void *stream, const double *src, double *dst, int ndim, const int64_t *shape,
                      const int64_t *sstride, const int64_t *dstride, int axis, const double *ss, int invert);
/* ev = <v, Mv>; Mv <- Mv - ev v; res2 = ||Mv||^2, one launch and one host read (contiguous n);
 * the residual of the step-size local solve (src/tt_als.py:1023-1030). */
int ttk_rayleigh_tail_sync(void *stream, const double *v, double *Mv, int64_t n, double *ev_out,
                           double *res2_out);
/* the same with (ev, ||Mv - ev v||^2) written to device memory out2[0..1] (no host wait): the
 * eigen-ALS sweep reads all local residuals of a half-sweep at once */
int ttk_rayleigh_tail_dev(void *stream, const double *v, double *Mv, int64_t n, double *out2);
/* dst = src * scales[i_axis] with the (<= 16) scales passed by value from the host: the per-block
 * column scaling / unscaling of the AMEn sweep (`src/tt_als.py:321-322,444-446`), no H2D copy. */
int ttk_scale_axis(void *stream, const double *src, double *dst, int ndim, const int64_t *shape,
                   const int64_t *sstride, const int64_t *dstride, int axis, const double *scales);
int ttk_fill(void *stream, double *dst, int64_t n, double value);
int ttk_add_diag(void *stream, double *A, int n, int lda, double value);

/* Reductions (strided up to 6-D), result copied to the host: sum(x*y), sum(x*x). */
int ttk_dot_nd_sync(void *stream, const double *x, const double *y, int ndim, const int64_t *shape,
                    const int64_t *xstride, const int64_t *ystride, double *result);
/* the same reduction into a device scalar, no host synchronisation (several norms of one sweep or
 * local solve are read back together) */
int ttk_dot_nd_dev(void *stream, const double *x, const double *y, int ndim, const int64_t *shape,
                   const int64_t *xstride, const int64_t *ystride, double *out);
/* batched sums of squares over `nb` contiguous slices of length n with stride `bstride`;
 * `out` is a device array of nb doubles (no sync). */
int ttk_sumsq_batched(void *stream, const double *x, int64_t n, int nb, int64_t bstride, double *out);
/* the same per-batch sums of squares over strided batches: element i (0 <= i < n) of batch b is
 * x[b*bstride + (i/inner)*ostride + i%inner], summed in i order exactly as ttk_sumsq_batched sums a
 * contiguous copy (per-block sums of a (r, B, n, R) core without the permuted copy). */
int ttk_sumsq_batched_strided(void *stream, const double *x, int64_t n, int nb, int64_t bstride, int64_t inner,
                              int64_t ostride, double *out);
/* copy `n` device doubles to the host (blocking) */
int ttk_read_sync(void *stream, const double *src, double *host_dst, int64_t n);
/* n doubles from pageable host memory to the device, asynchronously on the stream (staged through
 * a ring of pinned slots; the host buffer may be reused on return).  The eigen-ALS / AMEn random
 * draws (NumPy MT19937, `src/tt_als.py:534,580,1041-1053`) reach the device this way. */
int ttk_upload(void *stream, const double *host, double *dev, int64_t n);

/* ---------------------------------------------------------------------------------------
 * Small dense factorisations, one 256..1024-thread workgroup each (matrices staged in LDS
 * when they fit, L2-resident global scratch otherwise).  Row-major, leading dimension = cols.
 * ------------------------------------------------------------------------------------- */
/* thin SVD A(m,n) = U(m,k) diag(S) Vt(k,n), k = min(m,n), S descending; one-sided Jacobi.
 * Replaces scipy.linalg.svd(gesvd/gesdd) in `cy_src/tt_ops_cy.pyx:205-211,404,418`,
 * `src/tt_als.py:269-274,331,457,1024,1171` and friends. `work` >= ttk_svd_work(m,n) doubles. */
int64_t ttk_svd_work(int m, int n);
int ttk_svd(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt,
            double *work);
/* ttk_svd with a deflation tolerance for large unfoldings: the column-pivoted QR that precedes
 * the multi-workgroup Jacobi stops once the remaining Frobenius norm is <= defl; the deflated
 * directions get S = 0 and zero vectors.  Callers pass 1e-3 x their truncation threshold, so
 * the dropped energy (<= 1e-6 threshold^2) cannot change a `prune_singular_vals` decision
 * (`cy_src/tt_ops_cy.pyx:161-177`).  defl = 0: exact. */
int ttk_svd_tol(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt,
                double *work, double defl);
/* ttk_svd_tol followed by the host read of S (blocking): `s_host` receives the min(m,n) singular
 * values, as ttk_read_sync(S) would.  On the one-workgroup path the SVD kernel stores them into
 * host-coherent memory itself, so the host's wait follows the SVD with no read kernel between --
 * the rank decisions of the truncated-SVD sweeps (`cy_src/tt_ops_cy.pyx:200-222`,
 * `src/tt_als.py:269-274,457`) wait on exactly this. */
int ttk_svd_tol_read(void *stream, const double *A, int m, int n, double *U, double *S, double *Vt,
                     double *work, double defl, double *s_host);
/* min(m,n) <= 96: one-workgroup kernel (column-pivoted QR + one-sided Jacobi on R^T in LDS);
 * larger: the multi-workgroup path (pivoted QR launches + one launch per Jacobi round).
 * ttk_svd_set_big_threshold(p <= 2) forces the multi-workgroup path for every size (tests);
 * returns the previous setting. */
int ttk_svd_set_big_threshold(int p);
/* economic Householder QR A(m,n) = Q(m,k) R(k,n), k=min(m,n)  (scipy.linalg.qr economic,
 * `cy_src/tt_ops_cy.pyx:147-151`, `src/tt_als.py:358,482`). */
int64_t ttk_qr_work(int m, int n);
int ttk_qr(void *stream, const double *A, int m, int n, double *Q, double *R, double *work);
/* QRs with min(m,n) >= k whose working set exceeds LDS take the blocked multi-workgroup
 * Householder path (default 48); k <= 2 forces it (tests).  Returns the previous threshold. */
int ttk_qr_set_big_threshold(int k);
/* Cholesky (lower) in place on A(n,n); status TTK_ERR_NOT_PD like LAPACK potrf info>0
 * (`src/tt_ipm.py:204-207,300-303`). Blocks on the stream to return the status. */
int ttk_cholesky_sync(void *stream, double *A, int n);
/* n at or above which ttk_cholesky_sync / ttk_trsm_lower run the blocked multi-workgroup kernels
 * (32-column panels, fp64-MFMA trailing updates; default 96).  Returns the previous value. */
int ttk_dense_set_block_min(int n);
/* triangular solve with matrix RHS B(n,nrhs) in place: op(L) X = B, L lower (trans=0) or
 * L^T (trans=1) (`forward_backward_sub`, `src/tt_ipm.py:178-181`). */
int ttk_trsm_lower(void *stream, const double *L, int n, double *B, int nrhs, int ldb, int trans);
/* LU with partial pivoting in place (getrf) + rcond estimate (gecon, 1-norm, Hager/Higham);
 * `piv` device int[n]; returns TTK_ERR_SINGULAR on an exact zero pivot.  `rcond_out` host.
 * (`scipy.linalg.solve(assume_a='gen')` / `lu_factor`, `src/tt_ipm.py:215,320,323`)
 * rcond_out is dgecon's estimate, except when one comparison-matrix sweep already certifies that
 * estimate to be >= 1e-13 (1 / (||A||_1 max(M(L)^-T M(U)^-T e)) <= dgecon's value): then that
 * certified lower bound is returned and the estimator is skipped -- the value is then ONLY valid
 * for the LinAlgWarning test of the callers (rcond < eps), which decides identically either way.
 * The same holds for the rcond of ttk_dense_schur_solve.  Callers that log or compare the value
 * set the context knob TTK_KNOB_RCOND_EXACT = 1 (or env TTK_RCOND_EXACT=1): dgecon's estimate always. */
int ttk_lu_sync(void *stream, double *A, int n, int *piv, double *work, double *rcond_out);
/* solve with LU factors, B(n,nrhs) in place (getrs) */
int ttk_lu_solve(void *stream, const double *LU, int n, const int *piv, double *B, int nrhs, int ldb);
/* symmetric eigen-decomposition A(n,n) = W diag(ev) W^T, cyclic Jacobi, ev ascending,
 * W columns = eigenvectors (replaces ARPACK eigsh / lobpcg on the step-size local problems,
 * `src/tt_als.py:963-993,1069-1098,1308`). */
int64_t ttk_syev_work(int n);
int ttk_syev(void *stream, double *A, int n, double *ev, double *W, double *work);
/* one extreme eigenpair of a symmetric A(n,n) (which = 0: smallest, 1: largest): Householder
 * tridiagonalisation + Sturm multisection + inverse iteration, one launch.  ev: 1 device double,
 * vec: n device doubles (unit 2-norm).  A is not modified.  Replaces the `eigsh(which='SA'|'LA')`
 * calls of the step-size ALS (`src/tt_als.py:963-993` (_step_size_local_solve),
 * `:1069-1098`, `:1308` (_eigen_local_solve)). */
int64_t ttk_syev_extreme_work(int n);
/* 3 <= n <= 128 takes a latency-optimised LDS kernel (4 waves below n = 64, 16 waves above;
 * Sturm multisection on 4 waves; 3 barriers per reflector);
 * on = 0 routes every size through the general one-workgroup / multi-workgroup kernels (tests).
 * Returns the previous setting. */
int ttk_syev_set_small(int on);
/* Beyond the LDS kernels, n <= this limit (default and maximum 2048) runs the multi-workgroup
 * tridiagonalisation with ONE launch per Householder step (reflector rebuilt per block in LDS);
 * larger n (or limit 0) the two-launch variant.  Returns the previous limit. */
int ttk_syev_set_fused_max(int n);
/* diagnostic counters of the factorisation kernels (8 x u64: svd calls, svd sweeps, eig calls,
 * multisection rounds, ...); synchronous; reset != 0 zeroes them */
int ttk_debug_counters(unsigned long long *out, int reset);
/* phase timers of the one-workgroup SVD into the debug counters [4..7] (diagnostics) */
int ttk_svd_set_timing(int on);
int ttk_syev_extreme(void *stream, const double *A, int n, int which, double *ev, double *vec, double *work);

/* Schur-reduced local KKT operator of the iterative local solve (`MatVecWrapper` /
 * `IneqMatVecWrapper`, cy_src/lgmres_cy.pyx:203-331,379-510) as a handle.  `descs`: 5 (ineq = 0)
 * or 7 block descriptors of 36 int64 words each, in ttk_einsum's format for the local apply
 * 'lsr,smnS,LSR,rnR->lmL' (4 operands: XAX_k, A_k, XAX_k1, x with any pointer; has_out = 0):
 * B00, B01, B21, B22, B01 (read as its transpose 'lsr,smnS,LSR,lmL->rnR') [, B31, B33].
 * inv_I: m device doubles.  Handles belong to ctx (NULL: the calling thread's current context).
 * *handle = 0 when a block's descriptor does not describe the local apply (the caller keeps the
 * per-block path); blocks beyond the fused kernel's limits give a handle on the pairwise plans.  ttk_schur_apply: out = A v for v = [y; x (; t)] in 2
 * launches, the same operations (and rounding) as the per-block fused applies. */
int ttk_schur_build(ttk_ctx ctx, int ineq, int64_t m, const int64_t *descs, const double *inv_I,
                    int64_t *handle);
int ttk_schur_apply(ttk_ctx ctx, int64_t handle, const double *v, double *out);  /* on ctx's stream */
int ttk_schur_free(ttk_ctx ctx, int64_t handle);

/* ---------------------------------------------------------------------------------------
 * LGMRES building blocks (PETSc KSPLGMRES semantics, see oracle/petsc_lgmres.py):
 * one Arnoldi orthogonalisation + Hessenberg/Givens update per call.  V is (ldv x n)
 * row-major (vector j at V + j*n); `hh` (HH|HES|GRS|CC|SS packed, see ttk_lgmres.hip) lives
 * on the device; the new residual estimate and the breakdown flags are returned to the host
 * (blocking).  Replaces PETSc KSP lgmres (`src/tt_ipm.py:101-154`). */
/* res_out[2] = {new residual estimate |GRS(it+1)|, HH(it,it) after rotation};
 * flags_out[2] = {happy breakdown, DIVERGED_NULL (zero rotation norm)} */
int ttk_lgmres_arnoldi_sync(void *stream, double *V, int n, int it, double *hh, int max_k,
                            double haptol, double *res_out, int *flags_out);
/* Same step without a host read, for speculative chunks of Arnoldi steps between two host syncs
 * (the host's per-step PETSc convergence test, `src/tt_ipm.py:149-154`, replayed on the chunk's
 * records afterwards).  ctl (device, zeroed once per solve): ctl[0] = stop flag; step record at
 * ctl[1 + 5*slot] = {marker, res, happy breakdown, null rotation, HH(it,it)}.  The step sets the
 * stop flag when res <= ttol, res >= divtol, res is not finite, or on breakdown / null rotation;
 * every later step's kernels return at entry, leaving V/HH exactly at the stopping step. */
int ttk_lgmres_arnoldi_async(void *stream, double *V, int n, int it, double *hh, int max_k,
                             double haptol, double ttol, double divtol, double *ctl, int slot,
                             double marker);
/* Build the correction y = HH \ GRS (in place in GRS), temp = sum_j y_j basis_j where the
 * basis list is given as a device pointer array of `nvec` vectors; x += temp; aug_temp = temp. */
/* k Arnoldi steps it0 .. it0+k-1 of a chunk with the native Schur operator `schur`
 * (ttk_schur_build) as the matvec: V[it+1] = A V[it] then ttk_lgmres_arnoldi_async(slot q,
 * marker marker0 + q) -- the host loop's chunk without a host round trip per step. */
int ttk_lgmres_chunk(void *stream, int64_t schur, double *V, int n, int it0, int k, double *hh,
                     int max_k, double haptol, double ttol, double divtol, double *ctl, double marker0);
int ttk_lgmres_build(void *stream, double *hh, int max_k, int it, const double *const *basis,
                     int nvec, int n, double *x, double *aug_temp);
/* A*aug = V (HES y) / nrm over it_total+1 basis vectors (LGMRES augmentation bookkeeping). */
int ttk_lgmres_aug(void *stream, const double *hh, int max_k, int it_total, const double *V,
                   int n, double unused, const double *aug_temp, double *augvec, double *a_augvec);

/* (it+1)*n at or above which the Arnoldi / build / augmentation steps run as multi-workgroup
 * kernels (default 16384 elements); 0 forces them everywhere, INT_MAX disables them (tests).
 * Current context only (TTK_KNOB_LGMRES_MW_MIN).  Returns the previous threshold. */
int ttk_lgmres_set_mw_threshold(int elems);

/* Whole local KKT solve by LGMRES (PETSc KSPLGMRES semantics, `src/tt_ipm.py:101-162,249-266`):
 * solves A x = b from x0 = 0 with A the Schur operator `schur` (ttk_schur_build, the context's
 * handle table), restart/augment/rtol/max_it as the reference sets them (`src/tt_ipm.py:249-251`),
 * Arnoldi steps enqueued in speculative chunks of `chunk` steps with one host read per chunk.
 * info: PETSc convergence reason (2 rtol, 3 atol, -3 its, -2 null, -5 breakdown, -4 dtol, -9 nan),
 * iterations, last residual estimate, operator applications.  TTK_ERR_NOT_CONVERGED: HH(it,it) = 0
 * (PETSC_ERR_CONV_FAILED, the reference's exception path). */
typedef struct {
  int reason;
  int its;
  double res;
  int matvecs;
} ttk_lgmres_info;
int ttk_lgmres(ttk_ctx ctx, int64_t schur, const double *b, double *x, int64_t n, int restart, int augment,
               double rtol, int max_it, int chunk, ttk_lgmres_info *info);

/* ---------------------------------------------------------------------------------------
 * TT rounding in one call (SURVEY §8(b) `ttk_round`): replaces `tt_rank_reduce`
 * (cy_src/tt_ops_cy.pyx:179-226: right-to-left QR sweep `tt_rl_orthogonalise` :132-159, then the
 * left-to-right truncated-SVD sweep at eps/sqrt(d-1) with `prune_singular_vals` :161-177) and,
 * mode 1, the tracked sweep of `tt_psd_rank_reduce` / `tt_mask_rank_reduce` (:261-388: eps/2,
 * discarded energy accumulated; *tail_out = (sum of discarded sigma^2)^(1/(2d)), the factor the
 * caller adds as factor*I or factor*mask; NaN when the train was returned unchanged).
 * cores[k]: device, contiguous (r_k, inner[k], r_{k+1}) fp64, caller-owned, rewritten IN PLACE with
 * the rounded core (ranks never grow, so it fits); ranks[0..d]: in the input bond ranks
 * (ranks[0] = ranks[d] = 1), out the new ones.  Same launches as the Python sweep: bit-identical.
 * Host decisions read the singular values (one sync per bond). */
int ttk_round(ttk_ctx ctx, int d, double *const *cores, const int64_t *inner, int64_t *ranks, double eps, int mode,
              double *tail_out);

/* Zip-up products in one call (SURVEY §8(b) `ttk_zipup`; `tt_fast_matrix_vec_mul`,
 * `tt_fast_mat_mat_mul`, `tt_fast_hadamard`, cy_src/tt_ops_cy.pyx:391-502).  The device computes the
 * exact core-wise product (Kronecker bonds) and rounds it once at eps with ttk_round -- the same
 * represented tensor as the reference's SVD-swap zip-up to within the eps both truncate at
 * (DESIGN.md §3.1).  kind: 0 matvec  a (ra, m, n, Ra) x b (rb, n, Rb)        -> (ra rb, m, Ra Rb)
 *                         1 matmat  a (ra, m, k, Ra) x b (rb, k, n, Rb)     -> (ra rb, m, n, Ra Rb)
 *                         2 hadamard of vector trains (ra, i, Ra) o (rb, i, Rb)
 *                         3 hadamard of matrix trains (ra, i, j, Ra) o (rb, i, j, Rb)
 * modes[3k..3k+2] = the physical extents of core k: (m, n, -), (m, k, n), (i, -, -), (i, j, -).
 * a_ranks / b_ranks: d+1 bond ranks each.  out[k]: caller-owned contiguous buffers of the unrounded
 * product core's size, rewritten in place by the rounding (ranks never grow); out_ranks: d+1, the
 * rounded ranks.  eps <= 0 or d == 1: the exact product, unrounded. */
int ttk_zipup(ttk_ctx ctx, int kind, int d, const double *const *a, const int64_t *a_ranks,
              const double *const *b, const int64_t *b_ranks, const int64_t *modes, double eps,
              double *const *out, int64_t *out_ranks);

/* Dense Schur-complement local KKT solve in one call (SURVEY §8(b) `ttk_local_assemble` +
 * `ttk_dense_schur_solve`; the dense branch of `_ipm_local_solver`, src/tt_ipm.py:183-229):
 * assembles L_XI = B22 diag(inv_I), L_eq = B01, L_Z = B21 (each 'lsr,smnS,LSR->lmLrnR'), Cholesky of
 * L_Z, forward/backward substitutions, A = L_eq L_Z^-1 L_XI L_eq^T + B00 + 1e-11 I, LU with
 * dgecon, then back-substitutes Y, Z, X into sol (r, 3, n, R).  blk: the blocks (0,0), (0,1), (2,1),
 * (2,2) of the local operator -- XAX_k[key] (r, s, r), A_k[key] (s, n, n, S) with element strides,
 * XAX_k1[key] (R, S, R), all contiguous but A.  rhs (r, 3, n, R) and inv_I (r, n, R) contiguous.
 * Status: TTK_OK; TTK_ERR_NOT_PD (Cholesky failed: scipy LinAlgError), TTK_ERR_SINGULAR (exact
 * zero pivot), TTK_ILL_CONDITIONED (rcond < eps/2: LinAlgWarning) -- the reference then falls back
 * to its iterative solve (src/tt_ipm.py:224-229).  Same launches as the Python path: bit-identical.
 * rcond_out: as for ttk_lu_sync (a certified lower bound unless TTK_KNOB_RCOND_EXACT is set). */
typedef struct {
  const double *L, *A, *R;
  int64_t s, S, a_strides[4];
} ttk_local_block;
int ttk_dense_schur_solve(ttk_ctx ctx, int64_t r, int64_t n, int64_t R, const ttk_local_block *blocks,
                          const double *rhs, const double *inv_I, double *sol, double *rcond_out);

/* The inequality variant (the dense branch of `_ipm_local_solver_ineq`, src/tt_ipm.py:284-352):
 * L_Z = B21 (Cholesky), L_Z^-1 L_X with L_X = B22, L_eq = B01, T_op = B31, the two Schur levels
 * A = B00 + L_eq L_Z^-1 L_XI L_eq^T and D = B33 + T_op L_Z^-1 L_X + 1e-11 I, both LU-factored without
 * a condition check (scipy lu_factor), then Y, T, Z, X back-substituted into sol (r, 4, n, R).
 * blk: the blocks (0,0), (0,1), (2,1), (2,2), (3,1), (3,3) as for ttk_dense_schur_solve; rhs
 * (r, 4, n, R) and inv_I (r, n, R) contiguous.  Status: TTK_OK, TTK_ERR_NOT_PD, TTK_ERR_SINGULAR
 * (the reference's LinAlgError -> iterative fallback).  Same launches as the Python path. */
int ttk_dense_schur_solve_ineq(ttk_ctx ctx, int64_t r, int64_t n, int64_t R, const ttk_local_block *blocks,
                               const double *rhs, const double *inv_I, double *sol);

#ifdef __cplusplus
}
#endif
#endif /* TTK_H */
