"""CPU restatement of the reference's block-TT containers, AMEn sweeps and step-size ALS
(`src/tt_als.py`) -- TEST INFRASTRUCTURE, checker only."""
import time

import numpy as np
import scipy as scp
import scipy.linalg as sla
import scipy.sparse
import scipy.sparse.linalg

from . import tt as T
from .tt import einsum

# diagnostics (tools/decision_trace.py): a list receives one record per AMEn truncation rank scan
RANK_TRACE = None


def get_block(i, btt):
    """`src/tt_als.py:12-14`"""
    b = int(np.argmax([len(c.shape) for c in btt]))
    return list(btt[:b]) + [btt[b][:, i]] + list(btt[b + 1:])


class BlockVector:
    """`src/tt_als.py:16-57`"""

    def __init__(self):
        self.rows = {}

    def __setitem__(self, i, v):
        if not isinstance(v, list):
            raise ValueError("Each entry must be a list")
        self.rows[i] = v

    def get_row(self, i):
        return self.rows.get(i, None)

    def keys(self):
        return self.rows.keys()

    def core(self, k):
        return {i: v[k] for i, v in self.rows.items()}

    @property
    def norm(self):
        return np.sqrt(sum(T.inner(v, v) for v in self.rows.values()))

    def __sub__(self, other):
        out = BlockVector()
        for i in self.rows:
            out[i] = T.rank_reduce(T.sub(self.get_row(i), other.get_row(i)), 1e-12)
        return out


class BlockMatrix:
    """`src/tt_als.py:87-162`: data blocks + aliases + transpose couplings."""

    def __init__(self):
        self.data = {}
        self.aliases = {}
        self.transposes = {}

    def __setitem__(self, key, v):
        self.data[key] = v

    def __getitem__(self, key):
        return self.data.setdefault(key, [])

    def add_alias(self, k1, k2, is_transpose=False):
        (self.transposes if is_transpose else self.aliases)[k1] = k2

    def keys(self):
        return self.data.keys()

    def tkeys(self):
        return self.data.keys() | self.transposes.values()

    def block_product(self, x, op_tol, eps=1e-12):
        """`src/tt_als.py:132-155`"""
        res = BlockVector()

        def acc(i, tt):
            if i in res.keys():
                res[i] = T.rank_reduce(T.add(res.get_row(i), tt), eps)
            else:
                res[i] = tt

        for (i, j) in list(self.data.keys()):
            acc(i, mat_vec_mul(self.data[i, j], get_block(j, x), op_tol, eps))
            if (i, j) in self.transposes:
                k, t = self.transposes[i, j]
                acc(k, mat_vec_mul(T.transpose(self.data[i, j]), get_block(t, x), op_tol, eps))
            if (i, j) in self.aliases:
                k, t = self.aliases[i, j]
                acc(k, mat_vec_mul(self.data[i, j], get_block(t, x), op_tol, eps))
        return res

    def get_submatrix(self, ri, ci):
        sm = BlockMatrix()
        sm.data = {(i, j): v for (i, j), v in self.data.items() if i <= ri and j <= ci}
        sm.aliases = {k: v for k, v in self.aliases.items() if v[0] <= ri and v[1] <= ci}
        sm.transposes = {k: v for k, v in self.transposes.items() if v[0] <= ri and v[1] <= ci}
        return sm


class CoreView:
    """Per-core view of a BlockMatrix (`src/tt_als.py:165-250`)."""

    def __init__(self, bm, k):
        self.bm = bm
        self.k = k
        self.transposes = bm.transposes
        self.aliases = bm.aliases

    def __getitem__(self, key):
        return self.bm.data[key][self.k]

    def __iter__(self):
        return iter(self.bm.data)

    def keys(self):
        return self.bm.data.keys()

    def local_product(self, L, R, x):
        """`block_local_product` (`:190-200`)."""
        out = np.zeros_like(x, dtype=np.float64)
        for (i, j) in self.bm.data:
            A = self[i, j]
            out[:, i] += einsum("lsr,smnS,LSR,rnR->lmL", L[i, j], A, R[i, j], x[:, j])
            if (i, j) in self.transposes:
                k, t = self.transposes[i, j]
                out[:, k] += einsum("lsr,smnS,LSR,lmL->rnR", L[i, j], A, R[i, j], x[:, t])
            if (i, j) in self.aliases:
                k, t = self.aliases[i, j]
                out[:, k] += einsum("lsr,smnS,LSR,rnR->lmL", L[i, j], A, R[i, j], x[:, t])
        return out

    def _compressed(self, L, R, x, shape, teq, tL, tR):
        out = np.zeros(shape, dtype=np.float64)
        for (i, j) in self.bm.data:
            A = self[i, j]
            out[:, i] += einsum("lsr,smnS,LSR,rnR->lmL", L[i, j], A, R[i, j], x[:, j])
            if (i, j) in self.transposes:
                k, t = self.transposes[i, j]
                out[:, k] += einsum(teq, (L[k, t] if tL else L[i, j]), A, (R[k, t] if tR else R[i, j]), x[:, t])
            if (i, j) in self.aliases:
                k, t = self.aliases[i, j]
                out[:, k] += einsum("lsr,smnS,LSR,rnR->lmL", L[i, j], A, R[i, j], x[:, t])
        return out

    def compressed_product(self, ZL, ZR, x, shape):
        """`:202-212`"""
        return self._compressed(ZL, ZR, x, shape, "lsr,snmS,LSR,rnR->lmL", True, True)

    def lcompressed_product(self, ZL, XR, x, shape):
        """`:215-225`"""
        return self._compressed(ZL, XR, x, shape, "lsr,snmS,RSL,rnR->lmL", True, False)

    def rcompressed_product(self, XL, ZR, x, shape):
        """`:228-238`"""
        return self._compressed(XL, ZR, x, shape, "rsl,snmS,LSR,rnR->lmL", False, True)


def rhs_local_product(bcore, L, R, nrmsc, shape):
    """`TTBlockVectorView.block_local_product` (`src/tt_als.py:79-83`)."""
    out = np.zeros(shape, dtype=np.float64)
    for i, c in bcore.items():
        out[:, i] += einsum("br,bnB,BR->rnR", L[i], nrmsc * c, R[i])
    return out


def phi_bck_A(P, xl, A, xr):
    return einsum("LSR,lML,sMNS,rNR->lsr", P, xl, A, xr)


def phi_fwd_A(P, xl, A, xr):
    return einsum("lsr,lML,sMNS,rNR->LSR", P, xl, A, xr)


def phi_bck_rhs(P, b, x):
    return einsum("BR,bnB,rnR->br", P, b, x)


def phi_fwd_rhs(P, b, x):
    return einsum("br,bnB,rnR->BR", P, b, x)


def truncated_svd(m, k):
    """`src/tt_als.py:269-274` (default gesdd driver)."""
    u, s, v = sla.svd(m, full_matrices=False, check_finite=False, overwrite_a=True)
    return u[:, :k], s[:k].reshape(-1, 1) * v[:k]


def _block_scales(sol):
    return np.maximum(np.array([np.linalg.norm(sol[:, b]) for b in range(sol.shape[1])]), 1e-10
                      ).reshape(1, -1, 1, 1)


class _Ctx:
    pass


def _sweep(c, backward, swp, last, dsf):
    """Restatement of `_bck_sweep` (`src/tt_als.py:277-394`) and `_fwd_sweep` (`:397-522`)."""
    d, B, N = c.d, c.B, c.N
    rx, rz = c.rx, c.rz
    x, z = c.x, c.z
    amen = c.amen
    local_res = np.inf if swp == 0 else 0
    local_dx = np.inf if swp == 0 else 0
    order = range(d - 1, -1, -1) if backward else range(d)
    for k in order:
        Ak = CoreView(c.A, k)
        bk = c.b.core(k)
        solving = swp > 0 and not last
        if solving:
            prev = x[k]
            sol, res_old, res_new, rhs, nrhs, dsf = c.local_solver(
                c.XAX[k], Ak, c.XAX[k + 1], c.Xb[k], bk, c.Xb[k + 1], prev, 3 * d, not dsf)
            local_res = max(local_res, res_old)
            local_dx = max(np.linalg.norm(sol - prev) / np.linalg.norm(sol), local_dx)
            if amen:
                zsh = (rz[k], B, N[k], rz[k + 1])
                Az = Ak.compressed_product(c.ZAX[k], c.ZAX[k + 1], sol, zsh)
                rz_ = rhs_local_product(bk, c.Zb[k], c.Zb[k + 1], 1, zsh)
                rz_ -= Az
                if backward:
                    resz = np.reshape(rz_, (rz[k] * B, N[k] * rz[k + 1])).T
                else:
                    resz = np.transpose(rz_, (0, 2, 1, 3)).reshape(rz[k] * N[k], B * rz[k + 1])
            sc = _block_scales(sol)
        else:
            sol = x[k]
            sc = _block_scales(sol)
            if amen and not last:
                if backward:
                    resz = np.reshape(z[k], (rz[k] * B, N[k] * rz[k + 1])).T
                else:
                    resz = np.reshape(z[k].transpose(0, 2, 1, 3), (rz[k] * N[k], B * rz[k + 1]))
        if backward:
            mat = np.reshape(sc * sol, (rx[k] * B, N[k] * rx[k + 1])).T
        else:
            mat = np.reshape(np.transpose(sc * sol, (0, 2, 1, 3)), (rx[k] * N[k], B * rx[k + 1]))

        interior = (k > 0) if backward else (k < d - 1)
        if not interior:
            if backward:
                x[k] = np.reshape(mat.T, (rx[k], B, N[k], rx[k + 1])) / sc
                if amen and not last:
                    z[k] = np.reshape(resz.T, (rz[k], B, N[k], rz[k + 1])) / sc
            else:
                x[k] = np.reshape(mat, (rx[k], N[k], B, rx[k + 1])).transpose(0, 2, 1, 3) / sc
                if amen and not last:
                    z[k] = np.reshape(resz, (rz[k], N[k], B, rz[k + 1])).transpose(0, 2, 1, 3) / sc
            continue

        u, s, v = sla.svd(mat, full_matrices=False, check_finite=False, overwrite_a=True)
        v = s.reshape(-1, 1) * v
        if not backward:
            u = u.reshape(rx[k], N[k], -1)
            v = v.reshape(-1, B, rx[k + 1])
        if solving:
            trunc_lim = max(2 * c.trunc_tol, res_new)
            r0 = min(T.prune_singular_vals(s, c.eps), c.r_max)
            if backward:
                cur = np.reshape((u[:, :r0] @ v[:r0]).T, (rx[k], B, N[k], rx[k + 1]))
                res = Ak.local_product(c.XAX[k], c.XAX[k + 1], cur) - rhs
            else:
                cur = einsum("rbR,Rdk->rbdk", u[:, :, :r0], v[:r0])
                res = Ak.local_product(c.XAX[k], c.XAX[k + 1], np.transpose(cur, (0, 2, 1, 3))) - rhs
            r = r0
            rats = []
            for r in range(r0 - 1, 0, -1):
                if backward:
                    piece = np.reshape((u[:, None, r] @ v[None, r, :]).T, (rx[k], B, N[k], rx[k + 1]))
                else:
                    piece = einsum("rbR,Rdk->rdbk", u[:, :, None, r], v[None, r])
                res -= Ak.local_product(c.XAX[k], c.XAX[k + 1], piece)
                rats.append(float(np.linalg.norm(res) / nrhs))
                if rats[-1] > trunc_lim:
                    break
            r += 1
            if RANK_TRACE is not None:
                RANK_TRACE.append({"e": "rank", "k": int(k), "bwd": bool(backward), "r0": int(r0), "r": int(r),
                                   "lim": float(trunc_lim), "rat": rats})
            if backward:
                u = np.reshape(u[:, :r].T, (r, N[k], rx[k + 1]))
                v = v[:r].T.reshape(rx[k], B, r)
                if amen and not last:
                    sh = (rz[k], B, N[k], rx[k + 1])
                    Axz = Ak.lcompressed_product(c.ZAX[k], c.XAX[k + 1], cur, sh)
                    rxz = rhs_local_product(bk, c.Zb[k], c.Xb[k + 1], 1, sh)
                    rxz -= Axz
                    kr = min(c.kick_rank, rz[k] * B, N[k] * rx[k + 1])
                    uz, _ = truncated_svd(np.reshape(rxz, (rz[k] * B, N[k] * rx[k + 1])).T, kr)
                    uz = uz.T.reshape(kr, N[k], rx[k + 1])
                    u = np.concatenate((np.reshape(u, (r, N[k], rx[k + 1])), uz), axis=0)
                    u, Rm = sla.qr(u.reshape(-1, N[k] * rx[k + 1]).T, mode="economic",
                                   check_finite=False, overwrite_a=True)
                    u = u.T.reshape(-1, N[k], rx[k + 1])
                    v = einsum("Rdk,kr->Rdr", v, Rm.T[:v.shape[-1]])
                    r = u.shape[0]
            else:
                if amen:
                    sh = (rx[k], B, N[k], rz[k + 1])
                    Axz = Ak.rcompressed_product(c.XAX[k], c.ZAX[k + 1],
                                                 einsum("rbR,Rdk->rdbk", u[:, :, :r], v[:r]), sh)
                    rxz = rhs_local_product(bk, c.Xb[k], c.Zb[k + 1], 1, sh)
                    rxz = np.transpose(rxz - Axz, (0, 2, 1, 3))
                    kr = min(c.kick_rank, rx[k] * N[k], B * rz[k + 1])
                    uz, _ = truncated_svd(np.reshape(rxz, (rx[k] * N[k], B * rz[k + 1])), kr)
                    uz = np.reshape(uz, (rx[k], N[k], kr))
                    u = np.concatenate((u[:, :, :r], uz), axis=-1)
                    u, Rm = sla.qr(u.reshape(rx[k] * N[k], -1), mode="economic", check_finite=False,
                                   overwrite_a=True)
                    u = u.reshape(rx[k], N[k], -1)
                    v = einsum("rR,Rdk->rdk", Rm[:, :r], v[:r])
                    r = v.shape[0]
                else:
                    u = u[:, :, :r]
                    v = v[:r]
        else:
            r = min(T.prune_singular_vals(s, c.eps), c.r_max)
            if backward:
                u = np.reshape(u[:, :r].T, (r, N[k], rx[k + 1]))
                v = v[:r].T.reshape(rx[k], B, r)
            else:
                u = u[:, :, :r]
                v = v[:r]

        if backward:
            x[k] = u
            x[k - 1] = einsum("rdc,cbR->rbdR", x[k - 1], v) / sc
            rx[k] = r
            c.XAX[k] = {key: phi_bck_A(c.XAX[k + 1][key], x[k], Ak[key], x[k]) for key in Ak.keys()}
            c.Xb[k] = {i: phi_bck_rhs(c.Xb[k + 1][i], bk[i], x[k]) for i in bk}
        else:
            v = einsum("rbR,Rdk->rbdk", v, x[k + 1])
            x[k] = u
            x[k + 1] = v.reshape(r, B, N[k + 1], rx[k + 2]) / sc
            rx[k + 1] = r
            c.XAX[k + 1] = {key: phi_fwd_A(c.XAX[k][key], x[k], Ak[key], x[k]) for key in Ak.keys()}
            c.Xb[k + 1] = {i: phi_fwd_rhs(c.Xb[k][i], bk[i], x[k]) for i in bk}

        if amen and not last:
            kr = min(c.kick_rank, *resz.shape)
            uz, vz = truncated_svd(resz, kr)
            if backward:
                uz = uz.T.reshape(kr, N[k], rz[k + 1])
                vz = np.reshape(vz.T, (rz[k], B, kr))
                z[k] = uz
                z[k - 1] = einsum("rdc,cbR->rbdR", z[k - 1], vz) / sc
                rz[k] = uz.shape[0]
                zz = {key: phi_bck_A(c.ZAX[k + 1][key], z[k], Ak[key], x[k]) for key in Ak.keys()}
                zz.update({lt: phi_bck_A(c.ZAX[k + 1][lt], z[k], np.transpose(Ak[ij], (0, 2, 1, 3)), x[k])
                           for ij, lt in Ak.transposes.items()})
                c.ZAX[k] = zz
                c.Zb[k] = {i: phi_bck_rhs(c.Zb[k + 1][i], bk[i], z[k]) for i in bk}
            else:
                uz = np.reshape(uz, (rz[k], N[k], kr))
                vz = np.reshape(vz, (kr, B, rz[k + 1]))
                z[k] = uz
                z[k + 1] = einsum("rbR,Rdk->rbdk", vz, z[k + 1]) / sc
                rz[k + 1] = uz.shape[-1]
                zz = {key: phi_fwd_A(c.ZAX[k][key], z[k], Ak[key], x[k]) for key in Ak.keys()}
                zz.update({lt: phi_fwd_A(c.ZAX[k][lt], z[k], np.transpose(Ak[ij], (0, 2, 1, 3)), x[k])
                           for ij, lt in Ak.transposes.items()})
                c.ZAX[k + 1] = zz
                c.Zb[k + 1] = {i: phi_fwd_rhs(c.Zb[k][i], bk[i], z[k]) for i in bk}
    return local_res, local_dx, dsf


def block_amen(A, b, term_tol, r_max=100, eps=1e-12, nswp=22, x0=None, local_solver=None,
               kick_rank=2, amen=False, verbose=False, trace=None):
    """`tt_block_amen` (`src/tt_als.py:525-670`)."""
    B = int(np.max([k[0] for k in A.keys()])) + 1
    model = next(iter(b.rows.values()))
    xshape = model[0].shape[1:-1]

    def fresh():
        return T.normalise([np.random.randn(1, *c.shape[1:-1], 1) for c in model[:-1]]) + \
            [np.random.randn(1, B, *xshape, 1)]

    def block_idx(cores):
        ids = [i for i, c in enumerate(cores) if c.ndim == 4 and c.shape[1] == B]
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
    c.A, c.b = A, b
    c.x = x
    c.XAX = [{k: np.ones((1, 1, 1)) for k in A.keys()}] + [{k: None for k in A.keys()} for _ in range(d - 1)] + \
        [{k: np.ones((1, 1, 1)) for k in A.keys()}]
    c.Xb = [{k: np.ones((1, 1)) for k in b.keys()}] + [{k: None for k in b.keys()} for _ in range(d - 1)] + \
        [{k: np.ones((1, 1)) for k in b.keys()}]
    c.rx = np.array([1] + T.ranks(x) + [1])
    c.amen = amen
    c.z = c.ZAX = c.Zb = c.rz = None
    if amen:
        tk = A.tkeys()
        c.ZAX = [{k: np.ones((1, 1, 1)) for k in tk}] + [{k: None for k in tk} for _ in range(d - 1)] + \
            [{k: np.ones((1, 1, 1)) for k in tk}]
        c.Zb = [{k: np.ones((1, 1)) for k in b.keys()}] + [{k: None for k in b.keys()} for _ in range(d - 1)] + \
            [{k: np.ones((1, 1)) for k in b.keys()}]
        c.z = ([np.divide(1, np.prod(x[0].shape[1:-1]) * kick_rank ** 2) * np.random.randn(*x[0].shape[:-1], kick_rank)]
               + [np.divide(1, np.prod(cc.shape[1:-1]) * kick_rank ** 2) * np.random.randn(kick_rank, *cc.shape[1:-1], kick_rank)
                  for cc in x[1:-1]]
               + [np.divide(1, np.prod(x[-1].shape[1:-1]) * kick_rank ** 2) * np.random.randn(kick_rank, *x[-1].shape[1:])])
        c.rz = np.array([1] + T.ranks(c.z) + [1])
    c.local_solver = local_solver
    c.trunc_tol = term_tol / np.sqrt(d)
    c.eps, c.r_max, c.kick_rank = eps, r_max, kick_rank
    last = False
    final_res = np.inf
    dsf = False
    swp = 0
    for swp in range(nswp + 1):
        local_res, local_dx, dsf = _sweep(c, direction > 0, swp, last, dsf)
        if trace is not None:
            trace.append(("sweep", swp, float(local_res), list(map(int, c.rx[1:-1]))))
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
    return c.x, final_res


def restarted_block_amen(A, b, rank_restriction, op_tol, termination_tol=1e-3, eps=1e-11,
                         num_restarts=3, inner_m=10, x0=None, local_solver=None, verbose=False,
                         trace=None):
    """`tt_restarted_block_amen` (`src/tt_als.py:744-825`)."""
    if x0 is not None:
        dim = len(x0)
        x0 = T.rank_retraction(x0, [dim] * (dim - 1))

    def solve(rhs, rank, x0_, iters, kr):
        return block_amen(A, rhs, termination_tol, r_max=rank, eps=eps, nswp=iters, x0=x0_,
                          local_solver=local_solver, kick_rank=kr, amen=True, verbose=verbose, trace=trace)

    rhs = b
    orig = rhs.norm
    if orig < 0.5 * op_tol:
        raise RuntimeError(f"\n\tAbsolute tolerance already reached: {orig:4f} < {op_tol:4f}")
    x, res = solve(rhs, rank_restriction, x0, inner_m, 2)
    if res < termination_tol:
        return x, res
    rn = (rhs - A.block_product(x, 0.1 * op_tol)).norm
    if rn < termination_tol * orig or rn < orig:
        return x, res
    for _ in range(1, num_restarts):
        dim = len(x)
        x = T.rank_retraction(x, [2 * dim] * (dim - 1))
        x, res = solve(rhs, rank_restriction + 4, x, inner_m, 4)
        rn = (rhs - A.block_product(x, 0.1 * op_tol)).norm
        if rn < termination_tol * orig or rn < orig:
            return x, res
    raise RuntimeError(f"\n\tNumber of restarts exhausted, Relative Error = {rn / orig:3e}. "
                       "Consider increasing rank ceiling.")


# --------------------------------------------------------------------------------------------
# approximate / exact products (`src/tt_als.py:1502-1768`)
# --------------------------------------------------------------------------------------------

def approx_mat_mat_mul(A, D, x0=None, kick_rank=None, nswp=50, tol=1e-6):
    """`src/tt_als.py:1502-1628`"""
    if x0 is None:
        mr = np.maximum((np.array(T.ranks(A)) + np.array(T.ranks(D))) / 2, 2).astype(int)
        x = T.random_gaussian(list(mr), A[0].shape[1:-1])
    else:
        x = x0
        mr = np.array(T.ranks(x0))
    if kick_rank is None:
        kick_rank = np.maximum(((T.symmetric_powers_of_two(len(A) - 1) - mr) / (nswp / 2)), 2).astype(int)
    d = len(x)
    rx = np.array([1] + T.ranks(x) + [1])
    N = np.array([c.shape[1] for c in x])
    M = np.array([c.shape[2] for c in x])
    P = [np.ones((1, 1, 1))] + [None] * (d - 1) + [np.ones((1, 1, 1))]
    nAD = np.ones(d - 1)
    nrmsc = 1.0
    nx = np.ones(d - 1)
    tol = tol / np.sqrt(d)
    last = False
    for swp in range(nswp):
        mres = np.inf if swp == 0 else 0
        for k in range(d - 1, -1, -1):
            if swp > 0:
                prev = x[k]
                sol = einsum("rab,amkA,bknB,RAB->rmnR", P[k], A[k], D[k], P[k + 1]) * nrmsc
                mres = max(mres, np.linalg.norm(sol - prev) / max(np.linalg.norm(sol), 1e-8))
                sol = np.reshape(sol, (rx[k], N[k] * M[k] * rx[k + 1])).T
            else:
                sol = np.reshape(x[k], (rx[k], N[k] * M[k] * rx[k + 1])).T
            if k > 0:
                u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True,
                                  lapack_driver="gesvd")
                v = s.reshape(-1, 1) * v
                r = T.prune_singular_vals(s, tol)
                if not last:
                    u, v, r = T.add_kick_rank(u[:, :r], v[:r], kick_rank[k - 1])
                else:
                    u, v = u[:, :r], v[:r]
                nrmsc *= nx[k - 1] / nAD[k - 1]
                x[k] = np.reshape(u.T, (r, N[k], M[k], rx[k + 1]))
                x[k - 1] = np.tensordot(x[k - 1], v.T, axes=([3], [0]))
                nn = np.linalg.norm(x[k - 1])
                nx[k - 1] *= nn
                x[k - 1] /= nn
                rx[k] = r
                P[k] = einsum("RAB,amkA,bknB,rmnR->rab", P[k + 1], A[k], D[k], x[k])
                nrm = np.linalg.norm(P[k])
                nrm = nrm if nrm > 0 else 1.0
                P[k] /= nrm
                nAD[k - 1] = nrm
                nrmsc *= nAD[k - 1] / nx[k - 1]
            else:
                x[k] = np.reshape(sol, (rx[k], N[k], M[k], rx[k + 1]))
        if last:
            break
        if mres < tol or swp == nswp - 1:
            last = True
        mres = 0
        for k in range(d):
            prev = x[k]
            sol = einsum("rab,amkA,bknB,RAB->rmnR", P[k], A[k], D[k], P[k + 1]) * nrmsc
            mres = max(mres, np.linalg.norm(sol - prev) / max(np.linalg.norm(sol), 1e-8))
            sol = np.reshape(sol, (rx[k] * N[k] * M[k], rx[k + 1]))
            if k < d - 1:
                nrmsc *= nx[k] / nAD[k]
                u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True,
                                  lapack_driver="gesvd")
                v = s.reshape(-1, 1) * v
                r = T.prune_singular_vals(s, tol)
                if not last:
                    u, v, r = T.add_kick_rank(u[:, :r], v[:r, :], kick_rank[k])
                else:
                    u, v = u[:, :r], v[:r, :]
                x[k] = u.reshape(rx[k], N[k], M[k], r)
                x[k + 1] = np.tensordot(v, x[k + 1], axes=([1], [0])).reshape(r, N[k + 1], M[k + 1], rx[k + 2])
                nn = np.linalg.norm(x[k + 1])
                nx[k] *= nn
                x[k + 1] /= nn
                rx[k + 1] = r
                P[k + 1] = einsum("rab,amkA,bknB,rmnR->RAB", P[k], A[k], D[k], x[k])
                nrm = np.linalg.norm(P[k + 1])
                nrm = nrm if np.greater(nrm, 0) else 1.0
                P[k + 1] /= nrm
                nAD[k] = nrm
                nrmsc *= nAD[k] / nx[k]
            else:
                x[k] = np.reshape(sol, (rx[k], N[k], M[k], rx[k + 1]))
        if last:
            break
        if mres < tol:
            last = True
    nxs = np.exp(np.sum(np.log(nx)) / d)
    return [nxs * c for c in x]


def approx_mat_vec_mul(A, dv, x0=None, kick_rank=None, nswp=50, tol=1e-6):
    """`src/tt_als.py:1637-1762`"""
    if x0 is None:
        mr = np.maximum((np.array(T.ranks(A)) + np.array(T.ranks(dv))) / 2, 2).astype(int)
        x = T.random_gaussian(list(mr), (A[0].shape[2],))
    else:
        x = x0
        mr = np.array(T.ranks(x0))
    if kick_rank is None:
        kick_rank = np.maximum(((T.symmetric_powers_of_two(len(A) - 1) - mr) / (nswp / 2)), 2).astype(int)
    d = len(x)
    rx = np.array([1] + T.ranks(x) + [1])
    N = np.array([c.shape[1] for c in x])
    P = [np.ones((1, 1, 1))] + [None] * (d - 1) + [np.ones((1, 1, 1))]
    nAd = np.ones(d - 1)
    nrmsc = 1.0
    nx = np.ones(d - 1)
    tol = tol / np.sqrt(d)
    last = False
    for swp in range(nswp):
        mres = np.inf if swp == 0 else 0
        for k in range(d - 1, -1, -1):
            if swp > 0:
                prev = x[k]
                sol = einsum("rab,amkA,bkB,RAB->rmR", P[k], A[k], dv[k], P[k + 1]) * nrmsc
                mres = max(mres, np.linalg.norm(sol - prev) / max(np.linalg.norm(sol), 1e-8))
                sol = np.reshape(sol, (rx[k], N[k] * rx[k + 1])).T
            else:
                sol = np.reshape(x[k], (rx[k], N[k] * rx[k + 1])).T
            if k > 0:
                u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True,
                                  lapack_driver="gesvd")
                v = s.reshape(-1, 1) * v
                r = T.prune_singular_vals(s, tol)
                if not last:
                    u, v, r = T.add_kick_rank(u[:, :r], v[:r], kick_rank[k - 1])
                else:
                    u, v = u[:, :r], v[:r]
                nrmsc *= nx[k - 1] / nAd[k - 1]
                x[k] = np.reshape(u.T, (r, N[k], rx[k + 1]))
                x[k - 1] = np.tensordot(x[k - 1], v.T, axes=([2], [0]))
                nn = np.linalg.norm(x[k - 1])
                nx[k - 1] *= nn
                x[k - 1] /= nn
                rx[k] = r
                P[k] = einsum("RAB,amkA,bkB,rmR->rab", P[k + 1], A[k], dv[k], x[k])
                nrm = np.linalg.norm(P[k])
                nrm = nrm if nrm > 0 else 1.0
                P[k] /= nrm
                nAd[k - 1] = nrm
                nrmsc *= nAd[k - 1] / nx[k - 1]
            else:
                x[k] = np.reshape(sol, (rx[k], N[k], rx[k + 1]))
        if last:
            break
        if mres < tol or swp == nswp - 1:
            last = True
        mres = 0
        for k in range(d):
            prev = x[k]
            sol = einsum("rab,amkA,bkB,RAB->rmR", P[k], A[k], dv[k], P[k + 1]) * nrmsc
            mres = max(mres, np.linalg.norm(sol - prev) / max(np.linalg.norm(sol), 1e-8))
            sol = np.reshape(sol, (rx[k] * N[k], rx[k + 1]))
            if k < d - 1:
                nrmsc *= nx[k] / nAd[k]
                u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True,
                                  lapack_driver="gesvd")
                v = s.reshape(-1, 1) * v
                r = T.prune_singular_vals(s, tol)
                if not last:
                    u, v, r = T.add_kick_rank(u[:, :r], v[:r, :], kick_rank[k])
                else:
                    u, v = u[:, :r], v[:r, :]
                x[k] = u.reshape(rx[k], N[k], r)
                x[k + 1] = np.tensordot(v, x[k + 1], axes=([1], [0])).reshape(r, N[k + 1], rx[k + 2])
                nn = np.linalg.norm(x[k + 1])
                nx[k] *= nn
                x[k + 1] /= nn
                rx[k + 1] = r
                P[k + 1] = einsum("rab,amkA,bkB,rmR->RAB", P[k], A[k], dv[k], x[k])
                nrm = np.linalg.norm(P[k + 1])
                nrm = nrm if np.greater(nrm, 0) else 1.0
                P[k + 1] /= nrm
                nAd[k] = nrm
                nrmsc *= nAd[k] / nx[k]
            else:
                x[k] = np.reshape(sol, (rx[k], N[k], rx[k + 1]))
        if last:
            break
        if mres < tol:
            last = True
    nxs = np.exp(np.sum(np.log(nx)) / d)
    return [nxs * c for c in x]


def mat_mat_mul(m1, m2, op_tol, eps):
    """`src/tt_als.py:1631-1634`"""
    if np.max(np.array(T.ranks(m1)) * np.array(T.ranks(m2))) <= 40:
        return T.rank_reduce(T.fast_mat_mat_mul(m1, m2, eps), eps=op_tol)
    return approx_mat_mat_mul(m1, m2, tol=op_tol)


def mat_vec_mul(m, v, op_tol, eps):
    """`src/tt_als.py:1765-1768`"""
    if np.max(np.array(T.ranks(m)) * np.array(T.ranks(v))) <= 80:
        return T.rank_reduce(T.fast_matrix_vec_mul(m, v, eps), op_tol)
    return approx_mat_vec_mul(m, v, tol=op_tol)
