"""Block-TT containers, AMEn sweeps and product dispatch on the MI355X -- drop-in for
`src/tt_als.py:12-825,1502-1768` (same names and control flow; every dense step is a libttk
HIP kernel, the host keeps only the discrete decisions the reference takes).

Environment updates (`compute_phi_*`) and the local operator apply (`block_local_product` and
its compressed variants) are the core-contraction kernels of the path: each is a planned einsum
whose pairwise steps run on the fp64-MFMA offset-table GEMM."""
import time

import ctypes
import os

import numpy as np

from . import dev as D
from . import rng as _rng
from . import tt_ops as T
from .dev import einsum

APPLY = "lsr,smnS,LSR,rnR->lmL"
# diagnostics (tools/decision_trace.py): a list receives one record per AMEn truncation rank scan
RANK_TRACE = None
APPLY_T = "lsr,smnS,LSR,lmL->rnR"


def _tt_get_block(i, btt):
    """`src/tt_als.py:12-14`"""
    b = int(np.argmax([c.dim() for c in btt]))
    return list(btt[:b]) + [btt[b][:, i]] + list(btt[b + 1:])


class TTBlockVector:
    """`src/tt_als.py:16-57`"""

    def __init__(self):
        self._data = {}

    def __setitem__(self, i, v):
        if not isinstance(v, list):
            raise ValueError("Each entry must be a list")
        self._data[i] = v

    def get_row(self, i):
        return self._data.get(i, None)

    def keys(self):
        return self._data.keys()

    def values(self):
        return self._data.values()

    def __iter__(self):
        return iter(self._data)

    def core(self, k):
        return {i: v[k] for i, v in self._data.items()}

    @property
    def norm(self):
        # every block's <v, v> in one host read, summed on the host in block order as before
        return np.sqrt(sum(T.tt_scalars([("ip", v, v) for v in self._data.values()])))

    def __sub__(self, other):
        out = TTBlockVector()
        for i in self._data:
            out[i] = T.tt_rank_reduce(T.tt_sub(self.get_row(i), other.get_row(i)), 1e-12)
        return out


class TTBlockMatrix:
    """`src/tt_als.py:87-162`"""

    def __init__(self):
        self._data = {}
        self._aliases = {}
        self._transposes = {}

    def add_alias(self, k1, k2, is_transpose=False):
        (self._transposes if is_transpose else self._aliases)[k1] = k2

    def __getitem__(self, key):
        if isinstance(key, tuple) and len(key) == 2:
            return self._data.setdefault(key, [])
        if isinstance(key, int):
            return TTBlockMatrixView(self, key)
        raise KeyError(f"Invalid key format: {key}")

    def __setitem__(self, key, v):
        if not (isinstance(key, tuple) and len(key) == 2):
            raise KeyError(f"Invalid key format: {key}")
        self._data[key] = v

    def keys(self):
        return self._data.keys()

    def tkeys(self):
        return self._data.keys() | self._transposes.values()

    def __iter__(self):
        return iter(self._data)

    def block_product(self, x, op_tol, eps=1e-12):
        """`src/tt_als.py:132-155`"""
        res = TTBlockVector()

        def acc(i, tt):
            if i in res.keys():
                res[i] = T.tt_rank_reduce(T.tt_add(res.get_row(i), tt), eps)
            else:
                res[i] = tt

        for (i, j) in list(self._data.keys()):
            acc(i, tt_mat_vec_mul(self._data[i, j], _tt_get_block(j, x), op_tol, eps))
            if (i, j) in self._transposes:
                k, t = self._transposes[i, j]
                acc(k, tt_mat_vec_mul(T.tt_transpose(self._data[i, j]), _tt_get_block(t, x), op_tol, eps))
            if (i, j) in self._aliases:
                k, t = self._aliases[i, j]
                acc(k, tt_mat_vec_mul(self._data[i, j], _tt_get_block(t, x), op_tol, eps))
        return res

    def get_submatrix(self, ri, ci):
        sm = TTBlockMatrix()
        sm._data = {(i, j): v for (i, j), v in self._data.items() if i <= ri and j <= ci}
        sm._aliases = {k: v for k, v in self._aliases.items() if v[0] <= ri and v[1] <= ci}
        sm._transposes = {k: v for k, v in self._transposes.items() if v[0] <= ri and v[1] <= ci}
        return sm


class TTBlockMatrixView:
    """Per-core view (`src/tt_als.py:165-250`)."""

    def __init__(self, bm, k):
        self.bm = bm
        self.k = k
        self._transposes = bm._transposes
        self._aliases = bm._aliases

    def __getitem__(self, key):
        return self.bm._data[key][self.k]

    def __iter__(self):
        return iter(self.bm._data)

    def keys(self):
        return self.bm._data.keys()

    def block_local_product(self, L, R, x, out=None):
        """`block_local_product` (`:190-200`); accumulates into `out` when given.  The block applies
        run as one einsum batch (grouped launches per dependency level)."""
        if out is None:
            out = D.zeros(*x.shape)
        with D.einsum_batch():
            return self._block_local_product(L, R, x, out)

    def _block_local_product(self, L, R, x, out):
        items = []  # (equation, operands, x column, out column) in the reference's block order
        for (i, j) in self.bm._data:
            ops = [L[i, j], self[i, j], R[i, j]]
            items.append((0, ops, j, i))
            if (i, j) in self._transposes:
                k, t = self._transposes[i, j]
                items.append((1, ops, t, k))
            if (i, j) in self._aliases:
                k, t = self._aliases[i, j]
                items.append((0, ops, t, k))
        return D.einsum_cols((APPLY, APPLY_T), items, x, out)

    def _compressed(self, L, R, x, out, teq, tL, tR):
        with D.einsum_batch():
            return self._compressed_body(L, R, x, out, teq, tL, tR)

    def _compressed_body(self, L, R, x, out, teq, tL, tR):
        items = []
        for (i, j) in self.bm._data:
            A = self[i, j]
            ops = [L[i, j], A, R[i, j]]
            items.append((0, ops, j, i))
            if (i, j) in self._transposes:
                k, t = self._transposes[i, j]
                items.append((1, [L[k, t] if tL else L[i, j], A, R[k, t] if tR else R[i, j]], t, k))
            if (i, j) in self._aliases:
                k, t = self._aliases[i, j]
                items.append((0, ops, t, k))
        return D.einsum_cols((APPLY, teq), items, x, out)

    def compressed_block_local_product(self, ZL, ZR, x, out):
        """`:202-212` (accumulates into out)"""
        return self._compressed(ZL, ZR, x, out, "lsr,snmS,LSR,rnR->lmL", True, True)

    def lcompressed_block_local_product(self, ZL, XR, x, out):
        """`:215-225`"""
        return self._compressed(ZL, XR, x, out, "lsr,snmS,RSL,rnR->lmL", True, False)

    def rcompressed_block_local_product(self, XL, ZR, x, out):
        """`:228-238`"""
        return self._compressed(XL, ZR, x, out, "rsl,snmS,LSR,rnR->lmL", False, True)


def rhs_local_product(bcore, L, R, out, alpha=1.0):
    """`TTBlockVectorView.block_local_product` (`src/tt_als.py:79-83`), accumulated into out."""
    with D.einsum_batch():
        D.einsum_cols(("br,bnB,BR->rnR",), [(0, [L[i], c, R[i]], -1, i) for i, c in bcore.items()], out, out,
                      alpha=alpha, beta=1.0)
    return out


# Environment updates as the one-launch fused local-apply kernel: relabelled, the 4-operand chain
# 'LSR,lML,sMNS,rNR->lsr' is the apply 'lsr,smnS,LSR,rnR->lmL' on strided views (no copies), so one
# launch replaces the three pairwise GEMM steps (same contraction, association as the greedy plan
# of the apply; operands beyond the fused kernel's LDS/FLOP limits fall back to the pairwise plan).
FUSED_ENV = os.environ.get("TTIPM_FUSED_ENV", "1") == "1"
_APPLY = "lsr,smnS,LSR,rnR->lmL"


def _shapes(*ops):
    return tuple(tuple(o.shape) for o in ops)


def compute_phi_bck_A(P, xl, A, xr):
    """`src/tt_als.py:252-253`"""
    if FUSED_ENV:
        return einsum(_APPLY, xl, A.permute(1, 0, 3, 2), xr, P, fused="env",
                      algo=("LSR,lML,sMNS,rNR->lsr", _shapes(P, xl, A, xr)))
    return einsum("LSR,lML,sMNS,rNR->lsr", P, xl, A, xr)


def compute_phi_fwd_A(P, xl, A, xr):
    """`src/tt_als.py:256-257`"""
    if FUSED_ENV:
        return einsum(_APPLY, xl.permute(2, 1, 0), A.permute(1, 3, 0, 2), xr.permute(2, 1, 0), P, fused="env",
                      algo=("lsr,lML,sMNS,rNR->LSR", _shapes(P, xl, A, xr)))
    return einsum("lsr,lML,sMNS,rNR->LSR", P, xl, A, xr)


class _EnvBlock(ctypes.Structure):
    _fields_ = [("phi", ctypes.c_void_p), ("x", ctypes.c_void_p), ("A", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("phi_shape", ctypes.c_int64 * 3), ("x_shape", ctypes.c_int64 * 3),
                ("A_shape", ctypes.c_int64 * 4), ("y_shape", ctypes.c_int64 * 3), ("a_strides", ctypes.c_int64 * 4)]


NATIVE_ENV = os.environ.get("TTIPM_NATIVE_ENV", "1") == "1"
# _ttkbind.env_update and the address of ttk_env_update it calls (None: pack in Python)
_ENV_NATIVE = ((D._BIND, ctypes.cast(D.lib.ttk_env_update, ctypes.c_void_p).value)
               if D._BIND is not None and hasattr(D._BIND, "env_update") and D.DEV.type == "cuda" else (None, None))


def env_update_many(backward, items):
    """All environment updates of one core step in ONE library call (`ttk_env_update`; the same
    relabelled fused applies as compute_phi_*_A, recorded into one einsum batch).  items: list of
    (P, x, A, y) with P, x, y contiguous; returns the new environments in order."""
    if not (NATIVE_ENV and FUSED_ENV and D.DEV.type == "cuda") or \
            not all(P.is_contiguous() and x.is_contiguous() and y.is_contiguous() for P, x, A, y in items):
        f = compute_phi_bck_A if backward else compute_phi_fwd_A
        return [f(P, x, A, y) for P, x, A, y in items]
    if D.ALGO is None and _ENV_NATIVE[0] is not None:  # descriptors packed natively (same library call)
        D._stream()
        return _ENV_NATIVE[0].env_update(_ENV_NATIVE[1], D.ctx().value, bool(backward), items)
    arr = (_EnvBlock * len(items))()
    outs = []
    for e, (P, x, A, y) in zip(arr, items):
        o = D.empty(*((x.shape[0], A.shape[0], y.shape[0]) if backward else (x.shape[2], A.shape[3], y.shape[2])))
        outs.append(o)
        e.phi, e.x, e.A, e.y, e.out = P.data_ptr(), x.data_ptr(), A.data_ptr(), y.data_ptr(), o.data_ptr()
        e.phi_shape[:] = tuple(P.shape)
        e.x_shape[:] = tuple(x.shape)
        e.A_shape[:] = tuple(A.shape)
        e.y_shape[:] = tuple(y.shape)
        e.a_strides[:] = tuple(A.stride())
        if D.ALGO is not None:
            eq = "LSR,lML,sMNS,rNR->lsr" if backward else "lsr,lML,sMNS,rNR->LSR"
            D.count_algo(D.algo_flops(eq, _shapes(P, x, A, y)), what=eq)
    D._stream()
    D.check(D.lib.ttk_env_update(D.ctx(), int(backward), len(items), arr), "env_update")
    return outs


def compute_phi_bck_rhs(P, b, x):
    """`src/tt_als.py:260-261`"""
    return einsum("BR,bnB,rnR->br", P, b, x)


def compute_phi_fwd_rhs(P, b, x):
    """`src/tt_als.py:264-265`"""
    return einsum("br,bnB,rnR->BR", P, b, x)


def truncated_svd(m, k):
    """`src/tt_als.py:269-274`: returns (u[:, :k], s[:k] * v[:k])."""
    U, S, Vt, _ = D.svd(D.contig(m), host=False)
    return U[:, :k], einsum("r,rj->rj", S[:k], Vt[:k])


def _block_sumsq(sol):
    """per-block sums of squares of a (r, B, n, R) core, left on the device: one kernel reading the
    blocks in place (the sums of a contiguous (B, r, n, R) copy, bit for bit)."""
    r, B = sol.shape[0], sol.shape[1]
    out = D.empty(B)
    if not sol.is_contiguous():
        sol = D.clone(sol)
    inner = sol.shape[2] * sol.shape[3]
    D.check(D.lib.ttk_sumsq_batched_strided(D._stream(), sol.data_ptr(), r * inner, B, inner, inner, B * inner,
                                            out.data_ptr()), "sumsq")
    return out


def _scales(sol):
    """`np.maximum([||sol[:, b]||], 1e-10)` (`src/tt_als.py:321-322`) as the device sums of squares
    the scaling kernels turn into sc / 1/sc themselves (no host read)."""
    ss = _block_sumsq(sol)
    return ss, ss, ss


def _scale_blocks(t, ss, out=None):
    """t * sc[b] along the block axis 1 of a (r, B, n, R) tensor -> new tensor (or into `out`, any
    strides)."""
    return D.scale_axis_ss(t, 1, ss, invert=False, out=out)


def _div_blocks_bdim(t, ss, axis):
    """t * (1 / sc[b]) along the block axis `axis`."""
    return D.scale_axis_ss(t, axis, ss, invert=True)


class _Ctx:
    pass


def _sweep(c, backward, swp, last, dsf):
    """`_bck_sweep` (`src/tt_als.py:277-394`) / `_fwd_sweep` (`:397-522`) on the device."""
    d, B, N = c.d, c.B, c.N
    rx, rz = c.rx, c.rz
    x, z = c.x, c.z
    amen = c.amen
    local_res = np.inf if swp == 0 else 0
    local_dx = np.inf if swp == 0 else 0
    # ||sol - prev|| / ||sol|| per core: the dots stay on the device and are read once after the
    # sweep (local_dx only feeds the stopping test after it); the host formula is applied in order
    dx_buf = D.empty(2 * d) if (swp > 0 and not last) else None
    dx_seq = []
    order = range(d - 1, -1, -1) if backward else range(d)
    for k in order:
        Ak = c.A[k]
        bk = c.b.core(k)
        solving = swp > 0 and not last
        interior = (k > 0) if backward else (k < d - 1)

        def prep(sol, solved):
            """everything of the core step between the local solve and the truncation SVD"""
            resz = None
            if solved:
                if sol is not prev:
                    diff = D.axpby(prev, sol, -1.0, 1.0, 1.0)  # sol - prev, one launch (= clone + copy_)
                    j = sum(1 for t in dx_seq if t is not None)
                    D.dot_into(diff, diff, dx_buf[2 * j:2 * j + 1])
                    D.dot_into(sol, sol, dx_buf[2 * j + 1:2 * j + 2])
                    dx_seq.append(j)
                else:
                    dx_seq.append(None)
                if amen:
                    zsh = (rz[k], B, N[k], rz[k + 1])
                    rz_ = D.zeros(*zsh)
                    rhs_local_product(bk, c.Zb[k], c.Zb[k + 1], rz_)
                    Az = D.zeros(*zsh)
                    Ak.compressed_block_local_product(c.ZAX[k], c.ZAX[k + 1], sol, Az)
                    D.copy_(rz_, Az, -1.0, 1.0)
                    if backward:
                        resz = rz_.view(rz[k] * B, N[k] * rz[k + 1]).t()
                    else:
                        resz = D.clone(rz_.permute(0, 2, 1, 3)).view(rz[k] * N[k], B * rz[k + 1])
            elif amen and not last:
                if backward:
                    resz = D.contig(z[k]).view(rz[k] * B, N[k] * rz[k + 1]).t()
                else:
                    resz = D.clone(z[k].permute(0, 2, 1, 3)).view(rz[k] * N[k], B * rz[k + 1])
            sc, scd, inv = _scales(sol)
            if backward:
                scaled = _scale_blocks(sol, scd)
                mat = scaled.view(rx[k] * B, N[k] * rx[k + 1]).t()
            else:  # scaled straight into (r, n, B, R) storage: the forward unfolding needs no copy
                store = D.empty(rx[k], N[k], B, rx[k + 1])
                scaled = _scale_blocks(sol, scd, out=store.permute(0, 2, 1, 3))
                mat = store.view(rx[k] * N[k], B * rx[k + 1])
            return resz, inv, scaled, mat

        svd_out = None
        if solving:
            # the new local residual (`_ipm_local_solver`: keep prev if it got worse) comes back in
            # ONE read with the truncation SVD's singular values: the core step is enqueued on the
            # solver's solution, and redone on prev in the rare case the residual grew
            prev = x[k]
            kk = min(rx[k] * B, N[k] * rx[k + 1]) if backward else min(rx[k] * N[k], B * rx[k + 1])
            comb = D.empty(1 + (kk if interior else 0))
            sol, res_old, _, rhs, nrhs, dsf = c.local_solver(
                c.XAX[k], Ak, c.XAX[k + 1], c.Xb[k], bk, c.Xb[k + 1], prev, 3 * d, not dsf, res_out=comb[:1])
            local_res = max(local_res, res_old)
            resz, inv, scaled, mat = prep(sol, True)
            if interior:
                svd_out = D.svd(D.contig(mat), host=False, S_out=comb[1:])
            h = D.read(comb)
            res_new = D.norm_of(h[0]) / nrhs
            if res_old < res_new and sol is not prev:
                dx_seq.pop()
                sol = prev
                resz, inv, scaled, mat = prep(sol, True)
                svd_out = None
            elif interior:
                svd_out = svd_out[:3] + (h[1:],)
            res_new = min(res_old, res_new)
        else:
            sol = x[k]
            resz, inv, scaled, mat = prep(sol, False)

        if not interior:
            if backward:
                x[k] = _div_blocks_bdim(scaled, inv, 1)
                if amen and not last:
                    zz = D.contig(resz.t()).view(rz[k], B, N[k], rz[k + 1])
                    z[k] = _div_blocks_bdim(zz, inv, 1)
            else:
                x[k] = _div_blocks_bdim(scaled, inv, 1)
                if amen and not last:
                    zz = resz.view(rz[k], N[k], B, rz[k + 1]).permute(0, 2, 1, 3)
                    z[k] = _div_blocks_bdim(zz, inv, 1)
            continue

        U, S, Vt, s = D.svd(D.contig(mat)) if svd_out is None else svd_out
        v = einsum("r,rj->rj", S, Vt)  # s * v
        if not backward:
            u3 = U.view(rx[k], N[k], -1)
            v3 = v.view(-1, B, rx[k + 1])
        if solving:
            trunc_lim = max(2 * c.trunc_tol, res_new)
            r0 = min(T.prune_singular_vals(s, c.eps), c.r_max)
            if backward:
                cur = einsum("ik,kj->ji", U[:, :r0], v[:r0]).view(rx[k], B, N[k], rx[k + 1])
            else:
                cur = einsum("rbR,Rdk->rdbk", u3[:, :, :r0], v3[:r0])
            res = D.scaled(rhs, -1.0)
            Ak.block_local_product(c.XAX[k], c.XAX[k + 1], cur, out=res)
            r = r0
            # every candidate's product in one einsum batch, then the sequential residual updates and
            # norms in one scan (one host read); the break rule is replayed on the host unchanged
            cands = list(range(r0 - 1, 0, -1))
            if cands:
                negs = D.zeros(len(cands), *res.shape)
                with D.einsum_batch():
                    for q, rr in enumerate(cands):
                        if backward:
                            piece = einsum("i,j->ji", U[:, rr], v[rr]).view(rx[k], B, N[k], rx[k + 1])
                        else:
                            piece = einsum("rb,dk->rdbk", u3[:, :, rr], v3[rr])
                        Ak._block_local_product(c.XAX[k], c.XAX[k + 1], piece, negs[q])
                ss = D.rank_scan(res, negs)
                for q, rr in enumerate(cands):
                    r = rr
                    if D.norm_of(ss[q]) / nrhs > trunc_lim:
                        break
            r += 1
            if RANK_TRACE is not None:
                RANK_TRACE.append({"e": "rank", "k": int(k), "bwd": bool(backward), "r0": int(r0), "r": int(r),
                                   "lim": float(trunc_lim),
                                   "rat": [float(D.norm_of(ss[q]) / nrhs) for q in range(r0 - r + 1)] if cands else []})
            if backward:
                v_new = D.clone(v[:r].t()).view(rx[k], B, r)
                if not (amen and not last):
                    u_new = D.clone(U[:, :r].t()).view(r, N[k], rx[k + 1])
                if amen and not last:
                    sh = (rz[k], B, N[k], rx[k + 1])
                    rxz = D.zeros(*sh)
                    rhs_local_product(bk, c.Zb[k], c.Xb[k + 1], rxz)
                    Axz = D.zeros(*sh)
                    Ak.lcompressed_block_local_product(c.ZAX[k], c.XAX[k + 1], cur, Axz)
                    D.copy_(rxz, Axz, -1.0, 1.0)
                    kr = min(c.kick_rank, rz[k] * B, N[k] * rx[k + 1])
                    uz, _ = truncated_svd(rxz.view(rz[k] * B, N[k] * rx[k + 1]).t(), kr)
                    # [u_new; uz^T]^T = [U[:, :r], uz] built transposed in place (no clone of the
                    # truncated left factor, no transpose copy before the QR)
                    catT = D.empty(N[k] * rx[k + 1], r + kr)
                    D.copy_(catT[:, :r], U[:, :r])
                    D.copy_(catT[:, r:], uz)
                    Qm, Rm = D.qr(catT)
                    u_new = D.clone(Qm.t()).view(-1, N[k], rx[k + 1])
                    v_new = einsum("Rdk,rk->Rdr", v_new, Rm[:, :v_new.shape[-1]])
                    r = u_new.shape[0]
                u, vv = u_new, v_new
            else:
                if amen:
                    sh = (rx[k], B, N[k], rz[k + 1])
                    rxz = D.zeros(*sh)
                    rhs_local_product(bk, c.Xb[k], c.Zb[k + 1], rxz)
                    Axz = D.zeros(*sh)
                    Ak.rcompressed_block_local_product(c.XAX[k], c.ZAX[k + 1],
                                                       einsum("rbR,Rdk->rdbk", u3[:, :, :r], v3[:r]), Axz)
                    D.copy_(rxz, Axz, -1.0, 1.0)
                    rxzp = D.clone(rxz.permute(0, 2, 1, 3))
                    kr = min(c.kick_rank, rx[k] * N[k], B * rz[k + 1])
                    uz, _ = truncated_svd(rxzp.view(rx[k] * N[k], B * rz[k + 1]), kr)
                    cat = D.empty(rx[k] * N[k], r + kr)
                    D.copy_(cat[:, :r], u3[:, :, :r].reshape(rx[k] * N[k], r) if u3[:, :, :r].is_contiguous() else D.clone(u3[:, :, :r]).view(rx[k] * N[k], r))
                    D.copy_(cat[:, r:], uz)
                    Qm, Rm = D.qr(cat)
                    u = Qm.view(rx[k], N[k], -1)
                    vv = einsum("rR,Rdk->rdk", Rm[:, :r], v3[:r])
                    r = vv.shape[0]
                else:
                    u = u3[:, :, :r]
                    vv = v3[:r]
        else:
            r = min(T.prune_singular_vals(s, c.eps), c.r_max)
            if backward:
                u = D.clone(U[:, :r].t()).view(r, N[k], rx[k + 1])
                vv = D.clone(v[:r].t()).view(rx[k], B, r)
            else:
                u = u3[:, :, :r]
                vv = v3[:r]

        if backward:
            x[k] = D.contig(u)
            x[k - 1] = _div_blocks_bdim(einsum("rdc,cbR->rbdR", x[k - 1], vv), inv, 1)
            rx[k] = r
        else:
            nv = einsum("rbR,Rdk->rbdk", vv, x[k + 1])
            x[k] = D.contig(u)
            x[k + 1] = _div_blocks_bdim(nv.view(r, B, N[k + 1], rx[k + 2]), inv, 1)
            rx[k + 1] = r

        zk = None
        if amen and not last:
            kr = min(c.kick_rank, *resz.shape)
            uz, vz = truncated_svd(resz, kr)
            if backward:
                uzc = D.clone(uz.t()).view(kr, N[k], rz[k + 1])
                vzc = D.clone(vz.t()).view(rz[k], B, kr)
                z[k] = uzc
                z[k - 1] = _div_blocks_bdim(einsum("rdc,cbR->rbdR", z[k - 1], vzc), inv, 1)
                rz[k] = kr
            else:
                uzc = D.contig(uz).view(rz[k], N[k], kr)
                vzc = D.contig(vz).view(kr, B, rz[k + 1])
                z[k] = uzc
                z[k + 1] = _div_blocks_bdim(einsum("rbR,Rdk->rbdk", vzc, z[k + 1]), inv, 1)
                rz[k + 1] = kr
            zk = z[k]
        # every environment of the core step (XAX/Xb and, for AMEn, ZAX/Zb; src/tt_als.py:372-387,
        # 499-514) in one einsum batch: grouped launches instead of one launch per block
        src, dst = (k + 1, k) if backward else (k, k + 1)
        keys = list(Ak.keys())
        items = [(c.XAX[src][key], x[k], Ak[key], x[k]) for key in keys]
        zkeys = []
        if zk is not None:
            zkeys = keys + [lt for ij, lt in Ak._transposes.items()]
            items += [(c.ZAX[src][key], zk, Ak[key], x[k]) for key in keys]
            items += [(c.ZAX[src][lt], zk, Ak[ij].transpose(1, 2), x[k]) for ij, lt in Ak._transposes.items()]
        envs = env_update_many(backward, items)
        c.XAX[dst] = dict(zip(keys, envs[:len(keys)]))
        if zk is not None:
            c.ZAX[dst] = dict(zip(zkeys, envs[len(keys):]))
        rhs_env = compute_phi_bck_rhs if backward else compute_phi_fwd_rhs
        with D.einsum_batch():
            c.Xb[dst] = {i: rhs_env(c.Xb[src][i], bk[i], x[k]) for i in bk}
            if zk is not None:
                c.Zb[dst] = {i: rhs_env(c.Zb[src][i], bk[i], zk) for i in bk}
    if dx_seq:
        n_used = sum(1 for j in dx_seq if j is not None)
        vals = D.read(dx_buf[:2 * n_used]) if n_used else None
        for j in dx_seq:
            if j is None:
                local_dx = max(0.0, local_dx)
            else:
                local_dx = max(D.norm_of(vals[2 * j]) / D.norm_of(vals[2 * j + 1]), local_dx)
    return local_res, local_dx, dsf


def _ones3():
    return T._const("one111", np.ones((1, 1, 1)))


def _ones2():
    return T._const("one11", np.ones((1, 1)))


def tt_block_amen(block_A, block_b, term_tol, r_max=100, eps=1e-12, nswp=22, x0=None, local_solver=None,
                  kick_rank=2, amen=False, verbose=False):
    """`tt_block_amen` (`src/tt_als.py:525-670`)."""
    B = int(np.max([k[0] for k in block_A.keys()])) + 1
    model = next(iter(block_b.values()))
    xshape = tuple(model[0].shape[1:-1])

    def fresh():
        head = T.tt_normalise([D.from_numpy(_rng.R().randn(1, *c.shape[1:-1], 1)) for c in model[:-1]])
        return head + [D.from_numpy(_rng.R().randn(1, B, *xshape, 1))]

    def block_idx(cores):
        ids = [i for i, cc in enumerate(cores) if cc.dim() == 4 and cc.shape[1] == B]
        return ids[0] if len(ids) == 1 else None

    direction = 1
    if x0 is None:
        x = fresh()
    else:
        x = x0
        bi = block_idx(x)
        if bi is None:
            print("\tAttention: dropping warm start with invalid block-core layout; reinitializing TT guess.")
            x = fresh()
        elif bi == 0:
            direction = -1
        elif bi == len(x) - 1:
            direction = 1
        else:
            print(f"\tAttention: dropping warm start with block core at index {bi}; expected boundary core.")
            x = fresh()
    if verbose:
        t0 = time.time()
        tswp = t0
    c = _Ctx()
    c.N = [cc.shape[-2] for cc in x]
    c.d = d = len(c.N)
    c.B = B
    c.A, c.b = block_A, block_b
    c.x = x
    o3, o2 = _ones3(), _ones2()
    c.XAX = [{k: o3 for k in block_A.keys()}] + [{k: None for k in block_A.keys()} for _ in range(d - 1)] + \
        [{k: o3 for k in block_A.keys()}]
    c.Xb = [{k: o2 for k in block_b.keys()}] + [{k: None for k in block_b.keys()} for _ in range(d - 1)] + \
        [{k: o2 for k in block_b.keys()}]
    c.rx = np.array([1] + T.tt_ranks(x) + [1])
    c.amen = amen
    c.z = c.ZAX = c.Zb = c.rz = None
    if amen:
        tk = block_A.tkeys()
        c.ZAX = [{k: o3 for k in tk}] + [{k: None for k in tk} for _ in range(d - 1)] + [{k: o3 for k in tk}]
        c.Zb = [{k: o2 for k in block_b.keys()}] + [{k: None for k in block_b.keys()} for _ in range(d - 1)] + \
            [{k: o2 for k in block_b.keys()}]
        z0 = [np.divide(1, np.prod(x[0].shape[1:-1]) * kick_rank ** 2) * _rng.R().randn(*x[0].shape[:-1], kick_rank)]
        zm = [np.divide(1, np.prod(cc.shape[1:-1]) * kick_rank ** 2) * _rng.R().randn(kick_rank, *cc.shape[1:-1], kick_rank)
              for cc in x[1:-1]]
        zl = [np.divide(1, np.prod(x[-1].shape[1:-1]) * kick_rank ** 2) * _rng.R().randn(kick_rank, *x[-1].shape[1:])]
        c.z = [D.from_numpy(a) for a in z0 + zm + zl]
        c.rz = np.array([1] + T.tt_ranks(c.z) + [1])
    c.local_solver = local_solver
    c.trunc_tol = term_tol / np.sqrt(d)
    c.eps, c.r_max, c.kick_rank = eps, r_max, kick_rank
    last = False
    final_res = np.inf
    dsf = False
    swp = 0
    for swp in range(nswp + 1):
        local_res, local_dx, dsf = _sweep(c, direction > 0, swp, last, dsf)
        if last:
            break
        if local_res < term_tol or local_dx < eps or swp == nswp - 2:
            last = True
            final_res = local_res
        if verbose:
            print("\t===Finishing up===" if last else f"\t=====Sweep {swp + 1}=====")
            print(f'\tDirection {direction}')
            print(f'\tResidual {local_res:.3e}')
            print(f"\tTT-sol rank: {c.rx[1:-1]}")
            print(f"\tTime: {(time.time() - tswp):3f}s")
            tswp = time.time()
        direction *= -1
    if verbose:
        print("\n\t---Results---")
        print('\tSolution rank is', c.rx[1:-1])
        print(f'\tResidual {final_res:.3e}', )
        print('\tNumber of sweeps', swp)
        print(f'\tTime: {time.time() - t0:3f}s', flush=True)
    return c.x, final_res


def tt_restarted_block_amen(block_A, block_b, rank_restriction, op_tol, termination_tol=1e-3, eps=1e-11,
                            num_restarts=3, inner_m=10, x0=None, local_solver=None, verbose=False):
    """`tt_restarted_block_amen` (`src/tt_als.py:744-825`)."""
    if x0 is not None:
        dim = len(x0)
        x0 = T.tt_rank_retraction(x0, [dim] * (dim - 1))

    def solve(rhs, rank, x0_, iters, kr):
        return tt_block_amen(block_A, rhs, termination_tol, r_max=rank, eps=eps, nswp=iters, x0=x0_,
                             local_solver=local_solver, kick_rank=kr, amen=True, verbose=verbose)

    rhs = block_b
    orig = rhs.norm
    if orig < 0.5 * op_tol:
        raise RuntimeError(f"\n\tAbsolute tolerance already reached: {orig:4f} < {op_tol:4f}")
    x, res = solve(rhs, rank_restriction, x0, inner_m, 2)
    if res < termination_tol:
        if verbose:
            print(f"\n\tTerminated on local criterion, Relative Error < {termination_tol:4f}")
        return x, res
    rn = (rhs - block_A.block_product(x, 0.1 * op_tol)).norm
    if rn < termination_tol * orig or rn < orig:
        return x, res
    for _ in range(1, num_restarts):
        dim = len(x)
        x = T.tt_rank_retraction(x, [2 * dim] * (dim - 1))
        x, res = solve(rhs, rank_restriction + 4, x, inner_m, 4)
        rn = (rhs - block_A.block_product(x, 0.1 * op_tol)).norm
        if rn < termination_tol * orig or rn < orig:
            return x, res
    raise RuntimeError(f"\n\tNumber of restarts exhausted, Relative Error = {rn / orig:3e}. "
                       "Consider increasing rank ceiling.")


# ------------------------------------------------------------------ ALS approximate products
_APPROX_EQ = {  # (local solution, backward environment, forward environment)
    4: ("rab,amkA,bknB,RAB->rmnR", "RAB,amkA,bknB,rmnR->rab", "rab,amkA,bknB,rmnR->RAB"),
    3: ("rab,amkA,bkB,RAB->rmR", "RAB,amkA,bkB,rmR->rab", "rab,amkA,bkB,rmR->RAB"),
}


def _tt_approx_product(A, Dm, x0, kick_rank, nswp, tol, verbose):
    """Shared body of `tt_approx_mat_mat_mul` (`src/tt_als.py:1502-1628`) and
    `tt_approx_mat_vec_mul` (`:1637-1762`): ALS projection of the product A.Dm onto a TT with
    SVD truncation at tol/sqrt(d) and random kicks (host MT19937 draws in the reference's order);
    environments are normalised and the scale carried in `nrmsc` exactly as the reference does."""
    nd = Dm[0].dim()
    e_loc, e_bck, e_fwd = _APPROX_EQ[nd]
    if x0 is None:
        mr = np.maximum((np.array(T.tt_ranks(A)) + np.array(T.tt_ranks(Dm))) / 2, 2).astype(int)
        shape = tuple(A[0].shape[1:-1]) if nd == 4 else (A[0].shape[2],)
        x = T.tt_random_gaussian(list(mr), shape)
    else:
        x = list(x0)
        mr = np.array(T.tt_ranks(x0))
    if kick_rank is None:
        kick_rank = np.maximum(((T.symmetric_powers_of_two(len(A) - 1) - mr) / (nswp / 2)), 2).astype(int)
    d = len(x)
    rx = np.array([1] + T.tt_ranks(x) + [1])
    modes = [tuple(c.shape[1:-1]) for c in x]
    nmod = [int(np.prod(m)) for m in modes]
    o3 = _ones3()
    P = [o3] + [None] * (d - 1) + [o3]
    nAD = np.ones(d - 1)
    nrmsc = 1.0
    nx = np.ones(d - 1)
    tol = tol / np.sqrt(d)

    def local(k):
        return einsum(e_loc, P[k], A[k], Dm[k], P[k + 1], alpha=nrmsc)

    # relative changes: the two dots of each go to device slots and are read once per half-sweep
    # (only the running max decides anything, at the end of the half-sweep); the host formula of
    # D.norm is applied to the read values in call order, so mres is bit-identical
    rel_buf, rel_n = D.empty(2 * d), [0]

    def rel_change(sol, prev):
        diff = D.axpby(prev, sol, -1.0, 1.0, 1.0)  # sol - prev (= clone + copy_)
        i = rel_n[0]
        D.dot_into(diff, diff, rel_buf[2 * i:2 * i + 1])
        D.dot_into(sol, sol, rel_buf[2 * i + 1:2 * i + 2])
        rel_n[0] += 1

    def rel_max(m):
        if rel_n[0]:
            v = D.read(rel_buf[:2 * rel_n[0]])
            for i in range(rel_n[0]):
                m = max(m, float(np.sqrt(max(v[2 * i], 0.0))) / max(float(np.sqrt(max(v[2 * i + 1], 0.0))), 1e-8))
            rel_n[0] = 0
        return m

    def unit_and_env(t, Pk):
        """(t / ||t||, ||t||) and (Pk / nrm, nrm) of one core step: both norms in ONE host read (the
        environment Pk does not depend on t; same values as two D.norm calls)"""
        buf = D.empty(2)
        D.dot_into(t, t, buf[0:1])
        D.dot_into(Pk, Pk, buf[1:2])
        h = D.read(buf)
        nn, nrm = D.norm_of(h[0]), D.norm_of(h[1])
        nrm = nrm if nrm > 0 else 1.0
        return D.scaled(t, 1.0 / nn), nn, D.scaled(Pk, 1.0 / nrm), nrm

    last = False
    swp = 0
    mres = 0.0
    for swp in range(nswp):
        mres = np.inf if swp == 0 else 0
        for k in range(d - 1, -1, -1):
            if swp > 0:
                sol = local(k)
                rel_change(sol, x[k])
            else:
                sol = D.contig(x[k])
            if k > 0:
                mat = D.clone(sol.view(rx[k], nmod[k] * rx[k + 1]).t())
                U, S, Vt, s = D.svd(mat)
                v = einsum("r,rj->rj", S, Vt)
                r = T.prune_singular_vals(s, tol)
                if not last:
                    u, v, r = T.add_kick_rank(D.contig(U[:, :r]), D.contig(v[:r]), int(kick_rank[k - 1]))
                else:
                    u, v = U[:, :r], v[:r]
                nrmsc *= nx[k - 1] / nAD[k - 1]
                x[k] = D.clone(u.t()).view(r, *modes[k], rx[k + 1])
                prev = D.contig(x[k - 1]).view(-1, rx[k])
                t = einsum("ic,jc->ij", prev, v).view(rx[k - 1], *modes[k - 1], r)
                Pk = einsum(e_bck, P[k + 1], A[k], Dm[k], x[k])
                x[k - 1], nn, P[k], nrm = unit_and_env(t, Pk)
                nx[k - 1] *= nn
                rx[k] = r
                nAD[k - 1] = nrm
                nrmsc *= nAD[k - 1] / nx[k - 1]
            else:
                x[k] = D.contig(sol).view(rx[k], *modes[k], rx[k + 1])
        mres = rel_max(mres)
        if last:
            break
        if mres < tol or swp == nswp - 1:
            last = True
        mres = 0
        for k in range(d):
            sol = local(k)
            rel_change(sol, x[k])
            if k < d - 1:
                nrmsc *= nx[k] / nAD[k]
                U, S, Vt, s = D.svd(D.contig(sol).view(rx[k] * nmod[k], rx[k + 1]))
                v = einsum("r,rj->rj", S, Vt)
                r = T.prune_singular_vals(s, tol)
                if not last:
                    u, v, r = T.add_kick_rank(D.contig(U[:, :r]), D.contig(v[:r]), int(kick_rank[k]))
                else:
                    u, v = U[:, :r], v[:r]
                x[k] = D.contig(u).view(rx[k], *modes[k], r)
                nxt = D.contig(x[k + 1]).view(rx[k + 1], -1)
                t = einsum("ij,jk->ik", v, nxt).view(r, *modes[k + 1], rx[k + 2])
                Pk = einsum(e_fwd, P[k], A[k], Dm[k], x[k])
                x[k + 1], nn, P[k + 1], nrm = unit_and_env(t, Pk)
                nx[k] *= nn
                rx[k + 1] = r
                nAD[k] = nrm
                nrmsc *= nAD[k] / nx[k]
            else:
                x[k] = D.contig(sol).view(rx[k], *modes[k], rx[k + 1])
        mres = rel_max(mres)
        if last:
            break
        if mres < tol:
            last = True
        if verbose:
            print('\tStarting Sweep: %d' % swp)
            print(f'\tResidual {mres}')
            print(f"\tTT-sol rank: {T.tt_ranks(x)}", flush=True)
    if verbose:
        print(f"\t Solution rank is {rx[1:-1]}\n\t Residual {mres}\n\t Number of sweeps {swp + 1}", flush=True)
    nxs = float(np.exp(np.sum(np.log(nx)) / d))
    return [D.scaled(c, nxs) for c in x]


def tt_approx_mat_mat_mul(A, Dm, x0=None, kick_rank=None, nswp=50, tol=1e-6, verbose=False):
    """`src/tt_als.py:1502-1628`"""
    return _tt_approx_product(A, Dm, x0, kick_rank, nswp, tol, verbose)


def tt_approx_mat_vec_mul(A, d_vec, x0=None, kick_rank=None, nswp=50, tol=1e-6, verbose=False):
    """`src/tt_als.py:1637-1762`"""
    return _tt_approx_product(A, d_vec, x0, kick_rank, nswp, tol, verbose)


# ------------------------------------------------------------------ product dispatch (`:1631-1768`)
def tt_mat_mat_mul(m1, m2, op_tol, eps, verbose=False):
    """`src/tt_als.py:1631-1634`"""
    if np.max(np.array(T.tt_ranks(m1)) * np.array(T.tt_ranks(m2))) <= 40:
        return T.tt_rank_reduce(T.tt_fast_mat_mat_mul(m1, m2, eps), eps=op_tol)
    return tt_approx_mat_mat_mul(m1, m2, tol=op_tol, verbose=verbose)


def tt_mat_vec_mul(mat, vec, op_tol, eps, verbose=False):
    """`src/tt_als.py:1765-1768`"""
    if np.max(np.array(T.tt_ranks(mat)) * np.array(T.tt_ranks(vec))) <= 80:
        return T.tt_rank_reduce(T.tt_fast_matrix_vec_mul(mat, vec, eps), op_tol)
    return tt_approx_mat_vec_mul(mat, vec, tol=op_tol, verbose=verbose)
