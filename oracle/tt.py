"""CPU (NumPy/SciPy) restatement of the reference's TT algebra -- TEST INFRASTRUCTURE.

Checker for the MI355X path; never imported by the product package.  Each function cites the
reference line it restates.  Semantics kept on purpose:
  * `scale` rounds alpha to fp32 and scales ONE core chosen by `np.random.randint`
    (`cy_src/tt_ops_cy.pyx:94-114`), consuming the global MT19937 stream;
  * `normalise` truncates the radius to a C int (`cy_src/tt_ops_cy.pyx:524`);
  * rounding / orthogonalisation mutate the caller's list in place
    (`cy_src/tt_ops_cy.pyx:154-157,215-222`).
"""
from functools import lru_cache

import numpy as np
import scipy.linalg as sla

# --------------------------------------------------------------------------------------------
# einsum with a cached greedy path (reference: `src/tt_ops.py:22-28`, opt_einsum greedy).
# --------------------------------------------------------------------------------------------


# opt_einsum 3.4.0 greedy semantics (`oracle/opt_einsum_greedy.py`): NumPy's own greedy planner caps
# intermediates at the largest operand and then contracts the 4-operand local applies naively.
from . import opt_einsum_greedy as _oe  # noqa: E402


def _path_and_flops(eq, shapes):
    return None, _oe.flops(eq, shapes)


# algorithmic contraction FLOP counter: opt_einsum greedy convention per call
ALGO = None


def einsum(eq, *ops):
    if ALGO is not None:
        flops = _oe.flops(eq, tuple(o.shape for o in ops))
        ALGO["flops"] += flops
        ALGO["calls"] += 1
        if "by_eq" in ALGO:
            e = ALGO["by_eq"].setdefault(eq, [0, 0.0])
            e[0] += 1
            e[1] += flops
    return _oe.contract(eq, *ops)


# --------------------------------------------------------------------------------------------
# constructors / bookkeeping (`cy_src/tt_ops_cy.pyx:19-128`)
# --------------------------------------------------------------------------------------------

def identity(d):
    core = np.eye(2).reshape(1, 2, 2, 1)
    return [core] * d


def zero_matrix(d):
    core = np.zeros((1, 2, 2, 1))
    return [core] * d


def one_matrix(d):
    core = np.ones((1, 2, 2, 1))
    return [core] * d


def E(i, j):
    """`src/tt_ops.py:16-19`"""
    e = np.zeros((1, 2, 2, 1))
    e[:, i, j] += 1
    return e


def ranks(tt):
    """`cy_src/tt_ops_cy.pyx:82-92`"""
    return [int(c.shape[0]) for c in tt[1:]]


def transpose(tt):
    """`cy_src/tt_ops_cy.pyx:57-78`: swap the two physical axes from the first max-ndim core on."""
    k = int(np.argmax([np.ndim(c) for c in tt]))
    return list(tt[:k]) + [np.swapaxes(c, 1, 2) for c in tt[k:]]


def swap_all(tt):
    """`cy_src/tt_ops_cy.pyx:118-128`"""
    return [np.swapaxes(c, 0, -1) for c in tt[::-1]]


def scale(alpha, tt):
    """`cy_src/tt_ops_cy.pyx:94-114` (fp32 alpha, random core)."""
    n = len(tt)
    idx = np.random.randint(0, n)
    a32 = float(np.float32(alpha))
    out = list(tt)
    out[idx] = a32 * tt[idx]
    return out


def _block_diag(a, b):
    """`cy_src/tt_ops_cy.pyx:228-241`"""
    out = np.zeros((a.shape[0] + b.shape[0], *a.shape[1:-1], a.shape[-1] + b.shape[-1]))
    mid = tuple(slice(None) for _ in a.shape[1:-1])
    out[(slice(0, a.shape[0]),) + mid + (slice(0, a.shape[-1]),)] = a
    out[(slice(a.shape[0], None),) + mid + (slice(a.shape[-1], None),)] = b
    return out


def add(t1, t2):
    """`cy_src/tt_ops_cy.pyx:243-258`: rank-additive sum."""
    if len(t1) == 1:
        return [t1[0] + t2[0]]
    return ([np.concatenate((t1[0], t2[0]), axis=-1)]
            + [_block_diag(a, b) for a, b in zip(t1[1:-1], t2[1:-1])]
            + [np.concatenate((t1[-1], t2[-1]), axis=0)])


def sub(t1, t2):
    """`src/tt_ops.py:189-190`"""
    return add(t1, scale(-1, t2))


def inner(t1, t2):
    """`cy_src/tt_ops_cy.pyx:504-520`"""
    res = np.ones((1, 1))
    for c1, c2 in zip(t1, t2):
        tmp = np.tensordot(res, c1, axes=([0], [0]))
        if c1.ndim == 4:
            res = np.tensordot(tmp, c2, axes=([0, 1, 2], [0, 1, 2]))
        else:
            res = np.tensordot(tmp, c2, axes=([0, 1], [0, 1]))
    return float(res[0, 0])


def norm(tt):
    """`src/tt_ops.py:306-310`"""
    ip = inner(tt, tt)
    return float(np.sqrt(ip)) if ip > 0 else 0.0


def normalise(tt, radius=1):
    """`cy_src/tt_ops_cy.pyx:522-526` -- radius is a C int (truncated)."""
    factor = np.divide(int(radius), np.sqrt(inner(tt, tt)))
    return scale(factor, tt)


def random_gaussian(target_ranks, shape=(2,)):
    """`cy_src/tt_ops_cy.pyx:528-533`"""
    rk = [1] + list(target_ranks) + [1]
    cores = [np.divide(1, a * int(np.prod(shape)) * b) * np.random.randn(a, *shape, b)
             for a, b in zip(rk[:-1], rk[1:])]
    return normalise(cores)


def symmetric_powers_of_two(length):
    """`cy_src/tt_ops_cy.pyx:538-554`"""
    if length <= 0:
        return np.array([], dtype=np.int64)
    half = length // 2
    out = np.empty(length, dtype=np.int64)
    for i in range(half):
        out[i] = 1 << (i + 1)
    if length % 2:
        out[half] = 1 << (half + 1)
    for i in range(half):
        out[length - 1 - i] = out[i]
    return out


def add_kick_rank(u, v, r_add=2):
    """`cy_src/tt_ops_cy.pyx:557-578`"""
    old_r = u.shape[1]
    uk = np.random.randn(u.shape[0], r_add)
    q, rm = sla.qr(np.ascontiguousarray(np.concatenate((u, uk), axis=1)), mode="economic",
                   check_finite=False)
    return q, rm[:, :old_r] @ v, q.shape[1]


# --------------------------------------------------------------------------------------------
# orthogonalisation and rounding (`cy_src/tt_ops_cy.pyx:130-226,261-388`)
# --------------------------------------------------------------------------------------------

def rl_orthogonalise(tt):
    """`cy_src/tt_ops_cy.pyx:132-159` (in place, i = d-1 .. 1)."""
    d = len(tt)
    if d == 1:
        return tt
    for i in range(d - 1, 0, -1):
        si = tt[i].shape
        sm = tt[i - 1].shape
        q, r = sla.qr(tt[i].reshape(si[0], -1).T, mode="economic", check_finite=False)
        nr = r.shape[0]
        tt[i] = q.T.reshape(nr, *si[1:])
        lead = sm[:len(si) - 1]
        tt[i - 1] = (tt[i - 1].reshape(int(np.prod(lead)), si[0]) @ r.T).reshape(*lead, nr)
    return tt


def rl_orthogonalise_py(tt):
    """`src/tt_ops.py:30-42`: quirky variant that also runs i = 0 (R moves into the LAST core)."""
    d = len(tt)
    if d == 1:
        return tt
    for i in range(d - 1, -1, -1):
        si = tt[i].shape
        sm = tt[i - 1].shape
        q, r = sla.qr(tt[i].reshape(tt[i].shape[0], -1).T, mode="economic", check_finite=False)
        tt[i] = q.T.reshape(-1, *si[1:-1], si[-1])
        tt[i - 1] = (tt[i - 1].reshape(-1, r.shape[-1]) @ r.T).reshape(-1, *sm[1:-1], tt[i].shape[0])
    return tt


def prune_singular_vals(s, eps):
    """`cy_src/tt_ops_cy.pyx:161-177`"""
    if np.linalg.norm(s) == 0.0:
        return 1
    sc = np.cumsum(np.abs(s[::-1]) ** 2)[::-1]
    r = int(np.argmax(sc < eps ** 2))
    r = max(r, 1)
    if sc[-1] > eps ** 2:
        r = s.size
    return r


def _svd(a):
    return sla.svd(a, full_matrices=False, check_finite=False, overwrite_a=True,
                   lapack_driver="gesvd")


def _round_sweep(tt, eps, track_tail):
    """Shared left-to-right SVD sweep of `tt_rank_reduce` (`:197-224`) and the PSD/mask
    variants (`:283-318`, `:349-384`).  Returns the accumulated discarded energy."""
    d = len(tt)
    rank = 1
    tail = 0.0
    for idx in range(d - 1):
        ish = tt[idx].shape
        nsh = tt[idx + 1].shape
        mat = tt[idx].reshape(rank * int(np.prod(ish[1:-1], dtype=np.int32)), -1)
        u, s, vt = _svd(mat)
        if track_tail:
            sc = np.cumsum(np.abs(s[::-1]) ** 2)[::-1]
            nr = int(np.argmax(sc < eps ** 2))
            nr = max(nr, 1)
            if sc[-1] > eps ** 2:
                nr = s.shape[0]
            if nr < s.shape[0]:
                tail += sc[nr]
        else:
            nr = prune_singular_vals(s, eps)
        tt[idx] = u[:, :nr].reshape(rank, *ish[1:-1], nr)
        tt[idx + 1] = (s[:nr].reshape(-1, 1) * vt[:nr, :] @ tt[idx + 1].reshape(nsh[0], -1)
                       ).reshape(nr, *nsh[1:-1], -1)
        rank = nr
    return tail


def rank_reduce(tt, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:179-226`"""
    d = len(tt)
    rk = np.array([1] + ranks(tt) + [1])
    if d == 1 or np.all(rk == 1):
        return tt
    eps = eps / np.sqrt(d - 1)
    tt = rl_orthogonalise(tt)
    _round_sweep(tt, eps, False)
    return tt


def psd_rank_reduce(tt, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:261-325`: rounding + (discarded energy)^(1/2d) * I on every core."""
    d = len(tt)
    eps = eps / 2.0
    rk = np.array([1] + ranks(tt) + [1])
    if d == 1 or np.all(rk == 1):
        return tt
    eps = eps / np.sqrt(d - 1)
    tt = rl_orthogonalise(tt)
    tail = _round_sweep(tt, eps, True)
    factor = pow(tail, 1.0 / (2 * d))
    eye = factor * np.eye(tt[0].shape[1]).reshape(1, *tt[0].shape[1:-1], 1)
    return add(tt, [eye] * d)


def mask_rank_reduce(tt, mask, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:328-388`"""
    d = len(tt)
    eps = eps / 2.0
    rk = np.array([1] + ranks(tt) + [1])
    if d == 1 or np.all(rk == 1):
        return tt
    eps = eps / np.sqrt(d - 1)
    tt = rl_orthogonalise(tt)
    tail = _round_sweep(tt, eps, True)
    factor = pow(tail, 1.0 / (2 * d))
    return add(tt, [factor * c for c in mask])


def rank_retraction(tt, upper_ranks):
    """`src/tt_ops.py:132-152` (argpartition top-k, unsorted)."""
    tt = rl_orthogonalise_py(tt)
    rank = 1
    for idx, up in enumerate(upper_ranks):
        ish = tt[idx].shape
        nsh = tt[idx + 1].shape
        U, S, VT = _svd(tt[idx].reshape(rank * int(np.prod(ish[1:-1], dtype=int)), -1))
        a = np.abs(S)
        nr = min(up, len(a > 0))
        sel = np.argpartition(a, -nr)[-nr:]
        S, U, VT = S[sel], U[:, sel], VT[sel, :]
        tt[idx] = U.reshape(rank, *ish[1:-1], nr)
        tt[idx + 1] = (np.diag(S) @ VT @ tt[idx + 1].reshape(VT.shape[-1], -1)).reshape(nr, *nsh[1:-1], -1)
        rank = nr
    return tt


# --------------------------------------------------------------------------------------------
# zip-up products with SVD core swaps (`cy_src/tt_ops_cy.pyx:391-502`)
# --------------------------------------------------------------------------------------------

def swap_cores(a, b, eps):
    """`cy_src/tt_ops_cy.pyx:393-426`"""
    if a.ndim == 3:
        c = np.tensordot(a, b, axes=([2], [0])).transpose((0, 2, 1, 3))
        m = c.reshape(a.shape[0] * b.shape[1], -1)
        u, s, v = _svd(m)
        r = prune_singular_vals(s, eps)
        na = np.reshape(u[:, :r] * s[:r].reshape(1, -1), (a.shape[0], b.shape[1], -1))
        nb = np.reshape(v[:r, :], (-1, a.shape[1], b.shape[2]))
        return na, nb
    c = np.tensordot(a, b, axes=([3], [0])).transpose((0, 3, 4, 1, 2, 5))
    m = c.reshape(a.shape[0] * b.shape[1] * b.shape[2], -1)
    u, s, v = _svd(m)
    r = prune_singular_vals(s, eps)
    na = np.reshape(u[:, :r] * s[:r].reshape(1, -1), (a.shape[0], b.shape[1], b.shape[2], -1))
    nb = np.reshape(v[:r, :], (-1, a.shape[1], a.shape[2], b.shape[3]))
    return na, nb


def _bubble(cores, i, eps):
    for j in range(i, -1, -1):
        cores[j], cores[j + 1] = swap_cores(cores[j], cores[j + 1], eps)


def fast_matrix_vec_mul(mat, vec, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:428-447`"""
    d = len(mat)
    leps = eps / np.sqrt(d - 1) if d > 1 else eps
    cores = [np.transpose(c, (2, 1, 0)) for c in reversed(vec)]
    for i in range(d):
        cores[0] = np.tensordot(mat[d - i - 1], cores[0], axes=([3, 2], [0, 1]))
        if i != d - 1:
            _bubble(cores, i, leps)
    return cores


def fast_mat_mat_mul(m1, m2, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:449-464`"""
    d = len(m1)
    leps = eps / np.sqrt(d - 1) if d > 1 else eps
    cores = [np.transpose(c, (3, 1, 2, 0)) for c in reversed(m2)]
    for i in range(d):
        cores[0] = np.tensordot(m1[d - i - 1], cores[0], axes=([3, 2], [0, 1]))
        if i != d - 1:
            _bubble(cores, i, leps)
    return cores


def fast_hadamard(t1, t2, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:466-502`"""
    d = len(t1)
    leps = eps / np.sqrt(d - 1) if d > 1 else eps
    if t1[0].ndim == 4 and t2[0].ndim == 4:
        cores = [np.transpose(c, (3, 1, 2, 0)) for c in reversed(t2)]
        for i in range(d):
            tc = np.tensordot(t1[d - i - 1], cores[0], axes=([3], [0]))
            dg = np.diagonal(tc, axis1=1, axis2=3)
            dg = np.diagonal(dg, axis1=1, axis2=2)
            cores[0] = dg.transpose(0, 2, 3, 1)
            if i != d - 1:
                _bubble(cores, i, leps)
        return cores
    cores = [np.transpose(c, (2, 1, 0)) for c in reversed(t2)]
    for i in range(d):
        tc = np.tensordot(t1[d - i - 1], cores[0], axes=([2], [0]))
        dg = np.diagonal(tc, axis1=1, axis2=2)
        cores[0] = dg.transpose(0, 2, 1)
        if i != d - 1:
            _bubble(cores, i, leps)
    return cores


# --------------------------------------------------------------------------------------------
# Python-level TT helpers (`src/tt_ops.py`)
# --------------------------------------------------------------------------------------------

def merge_cores(tt):
    """`src/tt_ops.py:335-339`"""
    if len(tt[0].shape[1:-1]) == 1:
        return [einsum("kir,rsK->kisK", a, b) for a, b in zip(tt[:-1:2], tt[1::2])]
    return [einsum("kijr,rsdK->kisjdK", a, b) for a, b in zip(tt[:-1:2], tt[1::2])]


def reshape(tt, shape):
    """`src/tt_ops.py:330-333`"""
    if np.prod(shape) > np.prod(tt[0].shape[1:-1]):
        tt = merge_cores(tt)
    return [c.reshape(c.shape[0], *shape, c.shape[-1]) for c in tt]


def IkronM(tt):
    """`src/tt_ops.py:360-363`: I (x) M per core, (r,4,4,R)."""
    eye = np.eye(2).reshape(1, 2, 2, 1)
    return [einsum("rmnR,lijL->rlminjRL", eye, c).reshape(c.shape[0], 4, 4, c.shape[-1]) for c in tt]


def MkronI(tt):
    """`src/tt_ops.py:365-368`"""
    eye = np.eye(2).reshape(1, 2, 2, 1)
    return [einsum("rmnR,lijL->rlminjRL", c, eye).reshape(c.shape[0], 4, 4, c.shape[-1]) for c in tt]


def diag_op(tt, eps=1e-18):
    """`src/tt_ops.py:371-375`"""
    n = tt[0].shape[1] * tt[0].shape[2]
    eye = np.eye(n)
    basis = [einsum("ij,rjR->rijR", eye, c.reshape(c.shape[0], n, c.shape[3])) for c in tt]
    return rank_reduce(basis, eps)


def diag(vec, eps=1e-18):
    """`src/tt_ops.py:312-316`"""
    eye = np.eye(vec[0].shape[1])
    return rank_reduce([einsum("ij,rjR->rijR", eye, c) for c in vec], eps)


def entrywise_sum(tt):
    """`src/tt_ops.py:342-352`"""
    eq = "ab,aijm,bijn->mn" if tt[0].ndim == 4 else "ab,aim,bin->mn"
    one = np.ones((1, *tt[0].shape[1:-1], 1))
    res = np.array([[1.0]])
    for c in tt:
        res = einsum(eq, res, c, one)
    return float(np.sum(res))


def split_bonds(tt):
    """`src/tt_ops.py:247-265`"""
    out = []
    for core in tt:
        sh = core.shape
        k = len(sh) // 2
        u, s, vt = sla.svd(core.reshape(int(np.prod(sh[:k])), -1), full_matrices=False,
                           check_finite=False, overwrite_a=True)
        keep = np.asarray(np.abs(s) > 1e-18).nonzero()[0]
        if len(keep) == 0:
            keep = np.array([0])
        s, u, vt = s[keep], u[:, keep], vt[keep, :]
        out += [u.reshape(*sh[:k], len(s)), (np.diag(s) @ vt).reshape(len(s), *sh[k:])]
    return out


def tril_one_matrix(d):
    """`src/tt_ops.py:377-385`"""
    if d == 1:
        return [np.array([[1, 0], [1, 1]], dtype=float).reshape(1, 2, 2, 1)]
    one = np.ones((1, 2, 2, 1))
    zero = np.zeros((1, 2, 2, 1))
    return ([np.concatenate((E(1, 0), E(0, 0) + E(1, 1)), axis=-1)]
            + [np.concatenate((np.concatenate((one, E(1, 0)), axis=0),
                               np.concatenate((zero, E(0, 0) + E(1, 1)), axis=0)), axis=-1)
               for _ in range(d - 2)]
            + [np.concatenate((one, E(1, 0) + E(0, 0) + E(1, 1)), axis=0)])


def triu_one_matrix(d):
    """`src/tt_ops.py:387-395`"""
    if d == 1:
        return [np.array([[1, 1], [0, 1]], dtype=float).reshape(1, 2, 2, 1)]
    one = np.ones((1, 2, 2, 1))
    zero = np.zeros((1, 2, 2, 1))
    return ([np.concatenate((E(0, 1), E(0, 0) + E(1, 1)), axis=-1)]
            + [np.concatenate((np.concatenate((one, E(0, 1)), axis=0),
                               np.concatenate((zero, E(0, 0) + E(1, 1)), axis=0)), axis=-1)
               for _ in range(d - 2)]
            + [np.concatenate((one, E(0, 1) + E(0, 0) + E(1, 1)), axis=0)])


def tt_sum(*args, op_tol=1e-18, rank_reduce_=True):
    """`src/tt_ops.py:321-328`"""
    acc = args[0]
    for a in args[1:]:
        acc = rank_reduce(add(acc, a), op_tol) if rank_reduce_ else add(acc, a)
    return acc


def to_tensor(tt):
    """`src/tt_ops.py:192-196`"""
    t = tt[0]
    for c in tt[1:]:
        t = np.tensordot(t, c, axes=(-1, 0))
    return np.sum(t, axis=(0, -1))


def matrix_to_dense(mtt):
    """`src/tt_ops.py:211-217`"""
    if len(mtt) == 1:
        return np.squeeze(mtt)
    t = to_tensor(mtt)
    n = t.ndim
    axes = list(range(0, n - 1, 2)) + list(range(1, n, 2))
    return np.transpose(t, axes).reshape(int(np.prod(t.shape[:n // 2])), -1)


# --------------------------------------------------------------------------------------------
# random graph generator (`src/tt_ops.py:398-520`)
# --------------------------------------------------------------------------------------------

def _skewed_probabilities(n, skew=0.0):
    idx = np.linspace(0, 1, n)
    w = np.exp(-skew * idx)
    return w / w.sum()


def _diag_projector(basis, discarded, probs, limit=2):
    dim = len(basis)
    k = np.random.randint(dim) if dim > 0 else 0
    src = np.random.choice(dim, size=k, replace=False)
    t1 = np.random.choice(dim, size=k, replace=True, p=probs)
    t2 = np.random.choice(dim, size=k, replace=True, p=probs)
    p1 = np.eye(dim - 1)
    p2 = np.eye(dim - 1)
    upd = discarded.copy()
    for i, j1, j2 in zip(src, t1, t2):
        if i in discarded and j1 != 0 and j2 != 0:
            if len(upd) <= limit or (j1 in discarded) or (j2 in discarded):
                p1 += np.outer(basis[i], basis[j1] - basis[i])
                p2 += np.outer(basis[i], basis[j2] - basis[i])
                upd.discard(i)
                upd.add(j1)
                upd.add(j2)
        else:
            p1 += np.outer(basis[i], basis[j1] - basis[i])
            p2 += np.outer(basis[i], basis[j2] - basis[i])
    return p1, p2, upd


def _random_projector(basis, probs):
    dim = len(basis)
    if dim == 0:
        return np.array([[]])
    k = np.random.randint(dim)
    src = np.random.choice(dim, size=k, replace=False)
    tgt = np.random.choice(dim, size=k, replace=True, p=probs)
    p = np.eye(dim - 1)
    for i, j in zip(src, tgt):
        p += np.outer(basis[i], basis[j] - basis[i])
    return p


def random_binary_sym(d, rank, skew=5.0):
    if rank <= 0:
        return []
    q, _ = np.linalg.qr(np.random.randn(rank, rank), mode="reduced")
    basis = np.vstack((np.zeros(rank), q.T))
    probs = _skewed_probabilities(rank + 1, skew)
    bsz = rank + 1
    ii = np.random.choice(bsz, size=3, replace=True, p=probs)
    first = np.zeros((1, 4, rank))
    first[:, [0, 1, 2, 3], :] = basis[[ii[0], ii[1], ii[1], ii[2]]]
    discarded = set()
    if ii[0] != 0:
        discarded.add(ii[0])
    if ii[2] != 0:
        discarded.add(ii[2])
    cores = [first]
    if d <= 1:
        return cores
    for _ in range(d - 2):
        core = np.empty((rank, 4, rank))
        off = _random_projector(basis, probs)
        core[:, 1, :] = off
        core[:, 0, :], core[:, 3, :], discarded = _diag_projector(basis, discarded, probs, limit=rank)
        core[:, 2, :] = off
        cores.append(core)
    avail = sorted(list(set(range(bsz)) - discarded))
    last = np.zeros((rank, 4, 1))
    srt = sorted(avail)
    ortho = np.random.choice(srt, size=2, replace=True, p=(probs[srt]) / sum(probs[srt]))
    term = np.random.choice(bsz, size=1, replace=True, p=probs)
    fin = [ortho[0], term[0], term[0], ortho[1]]
    last[:, :, 0] = basis[fin].T
    cores.append(last)
    return cores


def random_graph(d, r, skew=-1.0, eps=1e-12, verbose=True):
    cur_rank = 0
    cur = None
    for _ in range(1, 1000):
        g = random_binary_sym(d, 2 * r, skew=skew)
        if norm(g) > 1e-12:
            g = rank_reduce(reshape(g, (2, 2)), 1e-12)
            mr = np.max(ranks(g))
            if cur_rank <= mr <= r:
                cur_rank = mr
                cur = g
            if cur_rank == r:
                break
    else:
        cur = [np.array([[0.0, 1.0], [1.0, 0.0]]).reshape(1, 2, 2, 1) for _ in range(d)]
    if verbose:
        print("===Terminated Graph Sampling=== rank: ", ranks(cur), flush=True)
    return cur
