"""TT algebra on the MI355X -- drop-in for the reference's `cy_src/tt_ops_cy.pyx` kernels and
`src/tt_ops.py` helpers (same names, argument meaning, in-place semantics and RNG coupling).

TT cores are fp64 device tensors; every arithmetic step is a libttk HIP kernel (dev.py).  The
only host<->device traffic is the singular values that drive truncation (`prune_singular_vals`
runs on the host, exactly as the reference decides ranks) and the scalars of inner products.

Semantics kept from the reference:
  * `tt_scale` rounds alpha to fp32 and scales ONE core chosen with `np.random.randint`
    (`cy_src/tt_ops_cy.pyx:94-114`) -- the host MT19937 stream is consumed identically;
  * `tt_normalise` truncates the radius to a C int (`cy_src/tt_ops_cy.pyx:524`);
  * `tt_rl_orthogonalise` / `tt_rank_reduce` overwrite the caller's list slots in place.
"""
from functools import reduce

import ctypes
import os

import numpy as np
from . import dev as D
from . import rng as _rng

def _const(name, arr):
    """Small constant cores, uploaded once per host thread (on that thread's stream)."""
    c = D._TL.consts
    t = c.get(name)
    if t is None:
        t = D.from_numpy(arr)
        c[name] = t
    return t


def _eye_core():
    return _const("eyecore", np.eye(2).reshape(1, 2, 2, 1))


def E(i, j):
    """`src/tt_ops.py:16-19`"""
    e = np.zeros((1, 2, 2, 1))
    e[:, i, j] += 1
    return _const(f"E{i}{j}", e)


def to_device(tt):
    return [D.from_numpy(c) for c in tt]


def to_host(tt):
    return [D.read(c) for c in tt]


# ------------------------------------------------------------------ constructors (`:19-53`)
def tt_identity(dim):
    c = _eye_core()
    return [c] * dim


def tt_zero_matrix(dim):
    c = _const("zero", np.zeros((1, 2, 2, 1)))
    return [c] * dim


def tt_one_matrix(dim):
    c = _const("one", np.ones((1, 2, 2, 1)))
    return [c] * dim


def tt_ranks(tt):
    """`cy_src/tt_ops_cy.pyx:82-92`"""
    return [int(c.shape[0]) for c in tt[1:]]


def tt_transpose(tt):
    """`cy_src/tt_ops_cy.pyx:57-78` (views)."""
    k = int(np.argmax([c.dim() for c in tt]))
    return list(tt[:k]) + [c.transpose(1, 2) for c in tt[k:]]


def tt_swap_all(tt):
    """`cy_src/tt_ops_cy.pyx:118-128` (views)."""
    return [c.transpose(0, -1) for c in tt[::-1]]


def tt_scale(alpha, tt):
    """`cy_src/tt_ops_cy.pyx:94-114`: fp32 alpha, one random core."""
    n = len(tt)
    idx = _rng.R().randint(0, n)
    out = list(tt)
    out[idx] = D.scaled(tt[idx], float(np.float32(alpha)))
    return out


DEV_JOIN = os.environ.get("TTIPM_DEV_JOIN", "1") == "1"


def _join(a, b, mode):
    """one-launch assembly (ttk_tt_join) for contiguous cores; None if not applicable."""
    if DEV_JOIN and a.is_contiguous() and b.is_contiguous() and a.dim() >= 2 and a.shape[1:-1] == b.shape[1:-1]:
        ra, Ra, rb, Rb = a.shape[0], a.shape[-1], b.shape[0], b.shape[-1]
        if (mode == 1 and ra != rb) or (mode == 2 and Ra != Rb):
            return None
        mid = int(np.prod(a.shape[1:-1])) if a.dim() > 2 else 1
        out = D.empty(ra if mode == 1 else ra + rb, *a.shape[1:-1], Ra if mode == 2 else Ra + Rb)
        D.check(D.lib.ttk_tt_join(D._stream(), a.data_ptr(), b.data_ptr(), out.data_ptr(), ra, Ra, rb, Rb, mid,
                                  mode), "tt_join")
        return out
    return None


def _block_diag(a, b):
    """`cy_src/tt_ops_cy.pyx:228-241`"""
    out = _join(a, b, 0)
    if out is not None:
        return out
    out = D.zeros(a.shape[0] + b.shape[0], *a.shape[1:-1], a.shape[-1] + b.shape[-1])
    D.copy_(out[:a.shape[0], ..., :a.shape[-1]], a)
    D.copy_(out[a.shape[0]:, ..., a.shape[-1]:], b)
    return out


def _cat(a, b, axis):
    out = _join(a, b, 2 if axis == 0 else 1)
    if out is not None:
        return out
    shp = list(a.shape)
    shp[axis] += b.shape[axis]
    out = D.empty(*shp)
    if axis == 0:
        D.copy_(out[:a.shape[0]], a)
        D.copy_(out[a.shape[0]:], b)
    else:
        D.copy_(out[..., :a.shape[-1]], a)
        D.copy_(out[..., a.shape[-1]:], b)
    return out


def tt_add(t1, t2):
    """`cy_src/tt_ops_cy.pyx:243-258`: rank-additive (block-diagonal) sum."""
    if len(t1) == 1:
        out = D.clone(t1[0])
        D.copy_(out, t2[0], 1.0, 1.0)
        return [out]
    return ([_cat(t1[0], t2[0], -1)] + [_block_diag(a, b) for a, b in zip(t1[1:-1], t2[1:-1])]
            + [_cat(t1[-1], t2[-1], 0)])


def tt_sub(t1, t2):
    """`src/tt_ops.py:189-190`"""
    return tt_add(t1, tt_scale(-1, t2))


def _inner_eq(nd):
    return "ab,aiA,biB->AB" if nd == 3 else "ab,aijA,bijB->AB"


def tt_inner_prod_dev(t1, t2):
    """Left-to-right contraction chain (`cy_src/tt_ops_cy.pyx:504-520`), result on the device."""
    res = _const("one11", np.ones((1, 1)))
    for c1, c2 in zip(t1, t2):
        res = D.einsum(_inner_eq(c1.dim()), res, c1, c2)
    return res


def tt_inner_prod(t1, t2):
    return float(D.read(tt_inner_prod_dev(t1, t2))[0, 0])


def tt_norm(tt):
    """`src/tt_ops.py:306-310`"""
    return norm_from_ip(tt_inner_prod(tt, tt))


def norm_from_ip(ip):
    """tt_norm's formula on a read-back <tt, tt>"""
    return float(np.sqrt(ip)) if ip > 0 else 0.0


def tt_scalars(specs):
    """Several TT scalars with ONE host read: ("ip", t1, t2) = tt_inner_prod(t1, t2), ("sum", tt) =
    tt_entrywise_sum(tt).  Each contraction chain is the one of the single-value function (same
    launches, same order); its last step writes straight into the chain's slot of one buffer."""
    buf = D.empty(max(len(specs), 1))
    with D.einsum_batch():  # the chains are independent: their steps grouped level by level
        _scalar_chains(specs, buf)
    return [float(v) for v in D.read(buf[:len(specs)])] if specs else []


def _scalar_chains(specs, buf):
    for i, sp in enumerate(specs):
        slot = buf[i:i + 1].view(1, 1)
        if sp[0] == "ip":
            t1, t2 = sp[1], sp[2]
            res = _const("one11", np.ones((1, 1)))
            for j, (c1, c2) in enumerate(zip(t1, t2)):
                res = D.einsum(_inner_eq(c1.dim()), res, c1, c2, out=slot if j == len(t1) - 1 else None)
        else:
            tt = sp[1]
            eq = "ab,aijm,bijn->mn" if tt[0].dim() == 4 else "ab,aim,bin->mn"
            one = _const("ones_" + "x".join(map(str, tt[0].shape[1:-1])), np.ones((1, *tt[0].shape[1:-1], 1)))
            res = _const("one11", np.ones((1, 1)))
            for j, c in enumerate(tt):
                res = D.einsum(eq, res, c, one, out=slot if j == len(tt) - 1 else None)


def tt_normalise(tt, radius=1):
    """`cy_src/tt_ops_cy.pyx:522-526` (int radius)."""
    factor = np.divide(int(radius), np.sqrt(tt_inner_prod(tt, tt)))
    return tt_scale(factor, tt)


def tt_random_gaussian(target_ranks, shape=(2,)):
    """`cy_src/tt_ops_cy.pyx:528-533` (host MT19937 draws, uploaded)."""
    rk = [1] + list(target_ranks) + [1]
    cores = [D.from_numpy(np.divide(1, a * int(np.prod(shape)) * b) * _rng.R().randn(a, *shape, b))
             for a, b in zip(rk[:-1], rk[1:])]
    return tt_normalise(cores)


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
    uk = D.from_numpy(_rng.R().randn(u.shape[0], r_add))
    q, rm = D.qr(_cat(u, uk, -1))
    return q, D.matmul(rm[:, :old_r], v), q.shape[1]


# ------------------------------------------------------------------ rounding (`:130-388`)
DEFL = 1e-3  # SVD deflation tolerance relative to a caller's truncation threshold


def prune_singular_vals(s, eps):
    """`cy_src/tt_ops_cy.pyx:161-177` -- host decision on the copied-back singular values."""
    if np.linalg.norm(s) == 0.0:
        return 1
    sc = np.cumsum(np.abs(s[::-1]) ** 2)[::-1]
    r = int(np.argmax(sc < eps ** 2))
    r = max(r, 1)
    if sc[-1] > eps ** 2:
        r = s.size
    return r


def _mat(t, rows):
    t = D.contig(t)
    return t.view(rows, -1)


def tt_rl_orthogonalise(tt):
    """`cy_src/tt_ops_cy.pyx:132-159` (in place, i = d-1 .. 1)."""
    d = len(tt)
    if d == 1:
        return tt
    for i in range(d - 1, 0, -1):
        si = tt[i].shape
        sm = tt[i - 1].shape
        Q, R = D.qr(D.contig(_mat(tt[i], si[0]).t()))
        nr = R.shape[0]
        tt[i] = D.clone(Q.t()).view(nr, *si[1:])
        lead = sm[:len(si) - 1]
        prev = D.contig(tt[i - 1]).view(int(np.prod(lead)), si[0])
        tt[i - 1] = D.einsum("ij,kj->ik", prev, R).view(*lead, nr)
    return tt


def tt_rl_orthogonalise_py(tt):
    """`src/tt_ops.py:30-42`: variant that also runs i = 0 (R moves into the LAST core)."""
    d = len(tt)
    if d == 1:
        return tt
    for i in range(d - 1, -1, -1):
        si = tt[i].shape
        sm = tt[i - 1].shape
        Q, R = D.qr(D.contig(_mat(tt[i], tt[i].shape[0]).t()))
        tt[i] = D.clone(Q.t()).view(-1, *si[1:-1], si[-1])
        prev = D.contig(tt[i - 1]).view(-1, R.shape[-1])
        tt[i - 1] = D.einsum("ij,kj->ik", prev, R).view(-1, *sm[1:-1], tt[i].shape[0])
    return tt


def _svd_step(tt, idx, rank, eps, track):
    ish = tt[idx].shape
    nsh = tt[idx + 1].shape
    mat = D.contig(tt[idx]).view(rank * int(np.prod(ish[1:-1])), -1)
    # deflation below 1e-3 x the truncation threshold cannot change the rank decision; the PSD /
    # mask variants (track) feed the discarded energy back, so they stay exact
    U, S, Vt, s = D.svd(mat, defl=0.0 if track else DEFL * eps)
    tail = 0.0
    if track:
        sc = np.cumsum(np.abs(s[::-1]) ** 2)[::-1]
        nr = int(np.argmax(sc < eps ** 2))
        nr = max(nr, 1)
        if sc[-1] > eps ** 2:
            nr = s.shape[0]
        if nr < s.shape[0]:
            tail = sc[nr]
    else:
        nr = prune_singular_vals(s, eps)
    tt[idx] = D.clone(U[:, :nr]).view(rank, *ish[1:-1], nr)
    nxt = D.contig(tt[idx + 1]).view(nsh[0], -1)
    tt[idx + 1] = D.einsum("r,rj,jk->rk", S[:nr], Vt[:nr], nxt).view(nr, *nsh[1:-1], -1)
    return nr, tail


NATIVE_ROUND = os.environ.get("TTIPM_NATIVE_ROUND", "1") == "1"


def _native_round(tt, eps, mode):
    """`ttk_round` (one library call per rounding, bit-identical to the Python sweep below).  The
    cores are copied first (the reference rebinds list entries and never writes the caller's
    arrays), the rounded cores are views of those copies.  Returns (tt, tail factor or None)."""
    d = len(tt)
    cs = D.clone_many(tt)
    mids = [tuple(c.shape[1:-1]) for c in tt]
    ptrs = (ctypes.c_void_p * d)(*[c.data_ptr() for c in cs])
    inner = (ctypes.c_int64 * d)(*[int(np.prod(m)) for m in mids])
    ranks = (ctypes.c_int64 * (d + 1))(*([tt[0].shape[0]] + [c.shape[-1] for c in tt]))
    tail = ctypes.c_double(0.0)
    D._stream()
    D.check(D.lib.ttk_round(D.ctx(), d, ptrs, inner, ranks, float(eps), mode, ctypes.byref(tail)), "round")
    out = [c.view(-1)[:ranks[k] * inner[k] * ranks[k + 1]].view(ranks[k], *mids[k], ranks[k + 1])
           for k, c in enumerate(cs)]
    tt[:] = out  # in place, like the reference's list mutation
    return tt, (None if np.isnan(tail.value) else tail.value)


def tt_rank_reduce(tt, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:179-226`: QR sweep + left-to-right truncated-SVD sweep."""
    d = len(tt)
    rk = [1] + tt_ranks(tt) + [1]
    if d == 1 or all(r == 1 for r in rk):
        return tt
    if NATIVE_ROUND and D.DEV.type == "cuda":
        return _native_round(tt, eps, 0)[0]
    eps = eps / np.sqrt(d - 1)
    tt = tt_rl_orthogonalise(tt)
    rank = 1
    for idx in range(d - 1):
        rank, _ = _svd_step(tt, idx, rank, eps, False)
    return tt


def _tail_rank_reduce(tt, eps):
    d = len(tt)
    rk = [1] + tt_ranks(tt) + [1]
    if d == 1 or all(r == 1 for r in rk):
        return tt, None
    if NATIVE_ROUND and D.DEV.type == "cuda":
        return _native_round(tt, eps, 1)
    eps = eps / 2.0
    eps = eps / np.sqrt(d - 1)
    tt = tt_rl_orthogonalise(tt)
    rank = 1
    tail = 0.0
    for idx in range(d - 1):
        rank, t = _svd_step(tt, idx, rank, eps, True)
        tail += t
    return tt, pow(tail, 1.0 / (2 * d))


def tt_psd_rank_reduce(tt, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:261-325`"""
    tt, factor = _tail_rank_reduce(tt, eps)
    if factor is None:
        return tt
    n = tt[0].shape[1]
    eye = D.from_numpy(factor * np.eye(n).reshape(1, *tt[0].shape[1:-1], 1))
    return tt_add(tt, [eye] * len(tt))


def tt_mask_rank_reduce(tt, mask, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:328-388`"""
    tt, factor = _tail_rank_reduce(tt, eps)
    if factor is None:
        return tt
    return tt_add(tt, [D.scaled(c, factor) for c in mask])


def tt_rank_retraction(tt, upper_ranks):
    """`src/tt_ops.py:132-152` (argpartition top-k on the host singular values)."""
    tt = tt_rl_orthogonalise_py(tt)
    rank = 1
    for idx, up in enumerate(upper_ranks):
        ish = tt[idx].shape
        nsh = tt[idx + 1].shape
        U, S, Vt, s = D.svd(D.contig(tt[idx]).view(rank * int(np.prod(ish[1:-1])), -1))
        a = np.abs(s)
        nr = min(up, len(a > 0))
        sel = np.argpartition(a, -nr)[-nr:]
        if np.array_equal(sel, np.arange(nr)):
            Us, Ss, Vs = U[:, :nr], S[:nr], Vt[:nr]
        else:  # unsorted top-k: gather the selected singular triplets with a 0/1 contraction
            Pn = np.zeros((len(s), nr))
            Pn[sel, np.arange(nr)] = 1.0
            P = D.from_numpy(Pn)
            Us = D.matmul(U, P)
            Ss = D.einsum("i,ij->j", S, P)
            Vs = D.einsum("ij,ik->jk", P, Vt)
        tt[idx] = D.contig(Us).view(rank, *ish[1:-1], nr)
        nxt = D.contig(tt[idx + 1]).view(Vs.shape[-1], -1)
        tt[idx + 1] = D.einsum("r,rj,jk->rk", Ss, Vs, nxt).view(nr, *nsh[1:-1], -1)
        rank = nr
    return tt


# ------------------------------------------------------------------ zip-up products (`:391-502`)
def swap_cores(a, b, eps):
    """`cy_src/tt_ops_cy.pyx:393-426`"""
    if a.dim() == 3:
        m = D.einsum("ijr,rkl->ikjl", a, b).view(a.shape[0] * b.shape[1], -1)
        U, S, Vt, s = D.svd(m, defl=DEFL * eps)
        r = prune_singular_vals(s, eps)
        na = D.einsum("ij,j->ij", U[:, :r], S[:r]).view(a.shape[0], b.shape[1], r)
        nb = D.clone(Vt[:r]).view(r, a.shape[1], b.shape[2])
        return na, nb
    m = D.einsum("ijkr,rlmn->ilmjkn", a, b).view(a.shape[0] * b.shape[1] * b.shape[2], -1)
    U, S, Vt, s = D.svd(m, defl=DEFL * eps)
    r = prune_singular_vals(s, eps)
    na = D.einsum("ij,j->ij", U[:, :r], S[:r]).view(a.shape[0], b.shape[1], b.shape[2], r)
    nb = D.clone(Vt[:r]).view(r, a.shape[1], a.shape[2], b.shape[3])
    return na, nb


def _bubble(cores, i, eps):
    for j in range(i, -1, -1):
        cores[j], cores[j + 1] = swap_cores(cores[j], cores[j + 1], eps)


def _zipup_matrix_vec_mul(mat, vec, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:428-447` as written (bubble zip-up); kept for the parity tests."""
    d = len(mat)
    leps = eps / np.sqrt(d - 1) if d > 1 else eps
    cores = [c.permute(2, 1, 0) for c in reversed(vec)]
    for i in range(d):
        cores[0] = D.einsum("amnA,Anr->amr", mat[d - i - 1], cores[0])
        if i != d - 1:
            _bubble(cores, i, leps)
    return cores


def _zipup_mat_mat_mul(m1, m2, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:449-464` as written (bubble zip-up); kept for the parity tests."""
    d = len(m1)
    leps = eps / np.sqrt(d - 1) if d > 1 else eps
    cores = [c.permute(3, 1, 2, 0) for c in reversed(m2)]
    for i in range(d):
        cores[0] = D.einsum("amkA,Aknr->amnr", m1[d - i - 1], cores[0])
        if i != d - 1:
            _bubble(cores, i, leps)
    return cores


def _zipup_hadamard(t1, t2, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:466-502` as written (bubble zip-up); kept for the parity tests."""
    d = len(t1)
    leps = eps / np.sqrt(d - 1) if d > 1 else eps
    if t1[0].dim() == 4 and t2[0].dim() == 4:
        cores = [c.permute(3, 1, 2, 0) for c in reversed(t2)]
        for i in range(d):
            cores[0] = D.einsum("aijA,Aijb->aijb", t1[d - i - 1], cores[0])
            if i != d - 1:
                _bubble(cores, i, leps)
        return cores
    cores = [c.permute(2, 1, 0) for c in reversed(t2)]
    for i in range(d):
        cores[0] = D.einsum("aiA,Aib->aib", t1[d - i - 1], cores[0])
        if i != d - 1:
            _bubble(cores, i, leps)
    return cores


# The reference's zip-up products contract each operator core into the reversed operand and
# bubble it through the processed cores with a truncated SVD per swap (eps/sqrt(d-1), absolute),
# i.e. d(d-1)/2 SVDs whose unfoldings live in a mode-permuted order: at maxcut_10 the bonds of
# those intermediates reach ~220 (888 x 1024 swap matrices) even though the product itself has
# rank <= rank_A * rank_x.  The device path computes the same product -- the exact core-wise
# (Kronecker-bond) contraction, truncated to the same absolute accuracy by one TT rounding at eps
# (QR sweep + d-1 truncated SVDs, `tt_rank_reduce`) -- so the represented tensor agrees with the
# zip-up's to within the eps both truncate at, without the mode-swapped intermediates.  The
# output ranks are the product's numerical ranks at eps (the zip-up's can only be larger, its
# per-swap truncation is not optimal); every hot call site rounds the result again
# (`tt_mat_vec_mul`, `tt_mat_mat_mul`, the residual / Y-update / centrality chains).
# TTIPM_ZIPUP=1 restores the bubble zip-up everywhere (parity experiments).
ZIPUP = os.environ.get("TTIPM_ZIPUP") == "1"


def _kron_round(cores, eps):
    if len(cores) > 1 and eps > 0:
        return tt_rank_reduce(cores, eps)
    return cores


NATIVE_ZIPUP = os.environ.get("TTIPM_NATIVE_ZIPUP", "1") == "1"


def _native_zipup(kind, a, b, eps, out_modes):
    """`ttk_zipup` (one library call: the core-wise products into fresh buffers + one in-place
    rounding; the same einsum plans and rounding launches as the Python composition below, so
    bit-identical to it).  out_modes[k]: the product core's physical shape."""
    d = len(a)
    ar = [a[0].shape[0]] + [c.shape[-1] for c in a]
    br = [b[0].shape[0]] + [c.shape[-1] for c in b]
    mids = []
    for x, y in zip(a, b):
        if kind == 0:
            mids += [x.shape[1], x.shape[2], 1]
        elif kind == 1:
            mids += [x.shape[1], x.shape[2], y.shape[2]]
        elif kind == 2:
            mids += [x.shape[1], 1, 1]
        else:
            mids += [x.shape[1], x.shape[2], 1]
    inner = [int(np.prod(m)) for m in out_modes]
    outs = [D.empty(ar[k] * br[k] * inner[k] * ar[k + 1] * br[k + 1]) for k in range(d)]
    ca = [D.contig(c) for c in a]
    cb = [D.contig(c) for c in b]
    P = ctypes.c_void_p
    I64 = ctypes.c_int64
    ranks = (I64 * (d + 1))()
    D._stream()
    D.check(D.lib.ttk_zipup(D.ctx(), kind, d, (P * d)(*[c.data_ptr() for c in ca]), (I64 * (d + 1))(*ar),
                            (P * d)(*[c.data_ptr() for c in cb]), (I64 * (d + 1))(*br), (I64 * (3 * d))(*mids),
                            float(eps), (P * d)(*[o.data_ptr() for o in outs]), ranks), "zipup")
    return [o[:ranks[k] * inner[k] * ranks[k + 1]].view(ranks[k], *out_modes[k], ranks[k + 1])
            for k, o in enumerate(outs)]


def _use_native_zipup():
    return NATIVE_ZIPUP and NATIVE_ROUND and D.DEV.type == "cuda"


def tt_fast_matrix_vec_mul(mat, vec, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:428-447`: mat (r_A,m,n,R_A) x vec (r,n,R) -> (r_A r, m, R_A R), rounded
    at eps (see the note above)."""
    if ZIPUP:
        return _zipup_matrix_vec_mul(mat, vec, eps)
    if _use_native_zipup():
        return _native_zipup(0, mat, vec, eps, [(a.shape[1],) for a in mat])
    cores = []
    for a, x in zip(mat, vec):
        ra, m, _, Ra = a.shape
        r, _, R = x.shape
        cores.append(D.einsum("amnA,rnR->armAR", a, x).view(ra * r, m, Ra * R))
    return _kron_round(cores, eps)


def tt_fast_mat_mat_mul(m1, m2, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:449-464`: core-wise matrix product, rounded at eps."""
    if ZIPUP:
        return _zipup_mat_mat_mul(m1, m2, eps)
    if _use_native_zipup():
        return _native_zipup(1, m1, m2, eps, [(a.shape[1], b.shape[2]) for a, b in zip(m1, m2)])
    cores = []
    for a, b in zip(m1, m2):
        ra, m, _, Ra = a.shape
        rb, _, n, Rb = b.shape
        cores.append(D.einsum("amkA,bknB->abmnAB", a, b).view(ra * rb, m, n, Ra * Rb))
    return _kron_round(cores, eps)


def tt_fast_hadamard(t1, t2, eps=1e-18):
    """`cy_src/tt_ops_cy.pyx:466-502`: core-wise Hadamard product, rounded at eps."""
    if ZIPUP:
        return _zipup_hadamard(t1, t2, eps)
    four = t1[0].dim() == 4 and t2[0].dim() == 4
    if _use_native_zipup() and (four or (t1[0].dim() == 3 and t2[0].dim() == 3)):
        return _native_zipup(3 if four else 2, t1, t2, eps, [tuple(a.shape[1:-1]) for a in t1])
    cores = []
    for a, b in zip(t1, t2):
        if four:
            cores.append(D.einsum("aijA,bijB->abijAB", a, b).view(a.shape[0] * b.shape[0], a.shape[1], a.shape[2],
                                                                  a.shape[3] * b.shape[3]))
        else:
            cores.append(D.einsum("aiA,biB->abiAB", a, b).view(a.shape[0] * b.shape[0], a.shape[1],
                                                             a.shape[2] * b.shape[2]))
    return _kron_round(cores, eps)


# ------------------------------------------------------------------ `src/tt_ops.py` helpers
def tt_merge_cores(tt):
    """`src/tt_ops.py:335-339`"""
    if tt[0].dim() == 3:
        return [D.einsum("kir,rsK->kisK", a, b) for a, b in zip(tt[:-1:2], tt[1::2])]
    return [D.einsum("kijr,rsdK->kisjdK", a, b) for a, b in zip(tt[:-1:2], tt[1::2])]


def tt_reshape(tt, shape):
    """`src/tt_ops.py:330-333` (views of contiguous cores)."""
    if np.prod(shape) > np.prod(tt[0].shape[1:-1]):
        tt = tt_merge_cores(tt)
    return [D.contig(c).view(c.shape[0], *shape, c.shape[-1]) for c in tt]


def tt_IkronM(tt):
    """`src/tt_ops.py:360-363`"""
    eye = _eye_core()
    return [D.einsum("rmnR,lijL->rlminjRL", eye, c).view(c.shape[0], 4, 4, c.shape[-1]) for c in tt]


def tt_MkronI(tt):
    """`src/tt_ops.py:365-368`"""
    eye = _eye_core()
    return [D.einsum("rmnR,lijL->rlminjRL", c, eye).view(c.shape[0], 4, 4, c.shape[-1]) for c in tt]


def tt_diag_op(tt, eps=1e-18):
    """`src/tt_ops.py:371-375`"""
    n = tt[0].shape[1] * tt[0].shape[2]
    eye = _const(f"eyemat{n}", np.eye(n))
    basis = [D.einsum("ij,rjR->rijR", eye, D.contig(c).view(c.shape[0], n, c.shape[3])) for c in tt]
    return tt_rank_reduce(basis, eps)


def tt_diag(vec, eps=1e-18):
    """`src/tt_ops.py:312-316`"""
    n = vec[0].shape[1]
    eye = _const(f"eyemat{n}", np.eye(n))
    return tt_rank_reduce([D.einsum("ij,rjR->rijR", eye, c) for c in vec], eps)


def tt_entrywise_sum(tt):
    """`src/tt_ops.py:342-352`"""
    eq = "ab,aijm,bijn->mn" if tt[0].dim() == 4 else "ab,aim,bin->mn"
    one = _const("ones_" + "x".join(map(str, tt[0].shape[1:-1])), np.ones((1, *tt[0].shape[1:-1], 1)))
    res = reduce(lambda r, c: D.einsum(eq, r, c, one), tt, _const("one11", np.ones((1, 1))))
    return float(np.sum(D.read(res)))


def tt_sum(*args, op_tol=1e-18, rank_reduce=True):
    """`src/tt_ops.py:321-328`"""
    acc = args[0]
    for a in args[1:]:
        acc = tt_rank_reduce(tt_add(acc, a), op_tol) if rank_reduce else tt_add(acc, a)
    return acc


def tt_split_bonds(tt):
    """`src/tt_ops.py:247-265` (problem generators only)."""
    out = []
    for core in tt:
        sh = core.shape
        k = len(sh) // 2
        U, S, Vt, s = D.svd(D.contig(core).view(int(np.prod(sh[:k])), -1))
        keep = np.nonzero(np.abs(s) > 1e-18)[0]
        if len(keep) == 0:
            keep = np.array([0])
        r = len(keep)
        assert np.array_equal(keep, np.arange(r))  # singular values are sorted descending
        out += [D.clone(U[:, :r]).view(*sh[:k], r), D.einsum("r,rj->rj", S[:r], Vt[:r]).view(r, *sh[k:])]
    return out


def _tril_host(d, upper):
    e = lambda i, j: (lambda z: (z.__setitem__((slice(None), i, j), 1.0), z)[1])(np.zeros((1, 2, 2, 1)))  # noqa: E731
    if d == 1:
        m = np.array([[1, 1], [0, 1]] if upper else [[1, 0], [1, 1]], dtype=float)
        return [m.reshape(1, 2, 2, 1)]
    one, zero = np.ones((1, 2, 2, 1)), np.zeros((1, 2, 2, 1))
    off = e(0, 1) if upper else e(1, 0)
    dg = e(0, 0) + e(1, 1)
    return ([np.concatenate((off, dg), axis=-1)]
            + [np.concatenate((np.concatenate((one, off), axis=0), np.concatenate((zero, dg), axis=0)), axis=-1)
               for _ in range(d - 2)]
            + [np.concatenate((one, off + dg), axis=0)])


def tt_tril_one_matrix(dim):
    """`src/tt_ops.py:377-385`"""
    return to_device(_tril_host(dim, False))


def tt_triu_one_matrix(dim):
    """`src/tt_ops.py:387-395`"""
    return to_device(_tril_host(dim, True))


def tt_to_tensor(tt):
    """`src/tt_ops.py:192-196` (host reconstruction, tests / small d only)."""
    t = D.read(tt[0])
    for c in tt[1:]:
        t = np.tensordot(t, D.read(c), axes=(-1, 0))
    return np.sum(t, axis=(0, -1))


def tt_matrix_to_matrix(mtt):
    """`src/tt_ops.py:211-217`"""
    if len(mtt) == 1:
        return np.squeeze(D.read(mtt[0]))
    t = tt_to_tensor(mtt)
    n = t.ndim
    axes = list(range(0, n - 1, 2)) + list(range(1, n, 2))
    return np.transpose(t, axes).reshape(int(np.prod(t.shape[:n // 2])), -1)
