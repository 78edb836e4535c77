"""Problem generators -- drop-in for `psd_system/{maxcut,corr_clust,graphm,max_stable_set}/<p>.py`
`create_problem(dim, rank)` (host-side problem creation, out of the timed region).

The random graph sampler (`src/tt_ops.py:398-520`) draws from the host NumPy MT19937 stream
exactly as the reference does; the resulting cores are uploaded and all TT arithmetic
(rounding, zip-up products, normalisation) runs on the device."""
import numpy as np

from . import dev as D
from . import tt_ops as T

E = T.E


# ------------------------------------------------------------------ random graph (`src/tt_ops.py:398-520`)
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


def tt_random_binary_sym_host(dim, rank, skew=5.0):
    """`src/tt_ops.py:455-502` (host cores)."""
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
    if dim <= 1:
        return cores
    for _ in range(dim - 2):
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


def tt_random_graph(dim, r, skew=-1.0, eps=1e-12, verbose=True):
    """`src/tt_ops.py:505-520`"""
    cur_rank = 0
    cur = None
    for _ in range(1, 1000):
        g = T.to_device(tt_random_binary_sym_host(dim, 2 * r, skew=skew))
        if T.tt_norm(g) > 1e-12:
            g = T.tt_rank_reduce(T.tt_reshape(g, (2, 2)), 1e-12)
            mr = np.max(T.tt_ranks(g))
            if cur_rank <= mr <= r:
                cur_rank = mr
                cur = g
            if cur_rank == r:
                break
    else:
        cur = [D.from_numpy(np.array([[0.0, 1.0], [1.0, 0.0]]).reshape(1, 2, 2, 1)) for _ in range(dim)]
    if verbose:
        print("===Terminated Graph Sampling=== rank: ", T.tt_ranks(cur), flush=True)
    return cur


def _ones_vec(dim):
    one = T._const("ones121", np.ones((1, 2, 1)))
    return [one] * dim


def _diag_constraint_op(dim):
    eye = T.tt_identity(dim)
    return T.tt_diag_op(eye), eye


# ------------------------------------------------------------------ maxcut (`psd_system/maxcut/maxcut.py`)
def maxcut_create_problem(dim, rank, verbose=True):
    """`psd_system/maxcut/maxcut.py:19-25`"""
    if verbose:
        print(f"Creating Problem for dim={dim}, rank={rank}...")
    scale = np.sqrt(dim)
    g = T.tt_rank_reduce(tt_random_graph(dim, rank, verbose=verbose))
    lap = T.tt_sub(T.tt_diag(T._zipup_matrix_vec_mul(g, _ones_vec(dim), 1e-12)), g)
    L, b = _diag_constraint_op(dim)
    lag_y = T.tt_diag_op(T.tt_sub(T.tt_one_matrix(dim), T.tt_identity(dim)))
    return (T.tt_reshape(T.tt_normalise(lap, radius=scale), (4,)), L,
            T.tt_reshape(T.tt_normalise(b, radius=scale), (4,)), lag_y)


# ------------------------------------------------------------------ corr_clust (`psd_system/corr_clust/corr_clust.py`)
def corr_clust_create_problem(dim, rank, verbose=True):
    """`psd_system/corr_clust/corr_clust.py:16-38`"""
    if verbose:
        print(f"Creating Problem for dim={dim}, rank={rank}...")
    scale = np.sqrt(dim)
    g = T.tt_rank_reduce(tt_random_graph(dim, rank, verbose=verbose), 1e-10)
    mg = T.tt_rank_reduce(tt_random_graph(dim, 1, verbose=verbose), 1e-10)
    sim = T.tt_rank_reduce(T._zipup_hadamard(g, mg, 1e-12), 1e-10)
    dis = T.tt_rank_reduce(T._zipup_hadamard(g, T.tt_sub(T.tt_one_matrix(dim), mg), 1e-12), 1e-10)
    lap = T.tt_sub(T.tt_diag(T._zipup_matrix_vec_mul(dis, _ones_vec(dim), 1e-12)), dis)
    obj = T.tt_rank_reduce(T.tt_add(sim, lap), 1e-10)
    if verbose:
        print("Actual graph TT-rank:", T.tt_ranks(g))
        print("Obj TT-rank:", T.tt_ranks(obj))
    L, b = _diag_constraint_op(dim)
    lag = {"y": T.tt_diag_op(T.tt_sub(T.tt_one_matrix(dim), T.tt_identity(dim))),
           "t": T.tt_diag_op(T.tt_sub(T.tt_one_matrix(dim), g))}
    return (T.tt_reshape(T.tt_normalise(obj, radius=scale), (4,)), L,
            T.tt_reshape(T.tt_normalise(b, radius=scale), (4,)), g, lag)


# ------------------------------------------------------------------ max_stable_set
def _new_core(c):
    return D.zeros(c.shape[0], 2, 2, c.shape[-1])


def _G_entrywise_mask_op(G):
    basis = []
    for gc in T.tt_split_bonds([D.clone(c) for c in G]):
        core = _new_core(gc)
        D.copy_(core[:, 0, 0], gc[:, 0])
        D.copy_(core[:, 1, 1], gc[:, 1])
        basis.append(core)
    return T.tt_rank_reduce(T.tt_reshape(basis, (4, 4)))


def _tr_constraint(dim):
    op = []
    for c in T.tt_split_bonds(T.to_device([np.eye(2).reshape(1, 2, 2, 1) for _ in range(dim)])):
        core = _new_core(c)
        D.copy_(core[:, 0], c)
        op.append(core)
    return T.tt_rank_reduce(T.tt_reshape(op, (4, 4))), [E(0, 0) for _ in range(dim)]


def max_stable_set_create_problem(dim, rank, verbose=True):
    """`psd_system/max_stable_set/max_stable_set.py:34-40`"""
    scale = np.sqrt(dim)
    G = T.tt_rank_reduce(tt_random_graph(dim, rank, verbose=verbose))
    obj = T.tt_one_matrix(dim)
    L, b = _tr_constraint(dim)
    L = T.tt_rank_reduce(T.tt_add(L, _G_entrywise_mask_op(G)))
    lag_y = T.tt_rank_reduce(T.tt_diag_op(T.tt_sub(T.tt_one_matrix(dim), T.tt_add(G, b))))
    return (T.tt_reshape(T.tt_normalise(obj, radius=scale), (4,)), L,
            T.tt_reshape(T.tt_normalise(b, radius=scale), (4,)), lag_y)


# ------------------------------------------------------------------ graphm (`psd_system/graphm/graphm.py`)
def _q_prefix():
    q = T._const("qprefix", np.array([[1.0, 0.0], [0.0, 0.0]]).reshape(1, 2, 2, 1))
    return [q, q]


def _split_diag(tt):
    return T.tt_diag(T.tt_split_bonds(tt))


def _partial_trace_op(bs, dim):
    op = _split_diag(T.tt_sub(T.tt_one_matrix(dim - bs), T.tt_identity(dim - bs)))
    blk = _split_diag(T.tt_identity(bs))
    return T.tt_reshape(T.tt_rank_reduce(_q_prefix() + op + blk), (4, 4))


def _placed(cores, which):
    out = []
    for i, c in enumerate(cores):
        core = _new_core(c)
        D.copy_(core[:, which(i)], c)
        out.append(core)
    return out


def _partial_J_trace_op(bs, dim):
    mt = T.tt_sub(T.tt_identity(dim - bs), [E(0, 0) for _ in range(dim - bs)])
    op0 = _split_diag(mt) + _placed(T.tt_split_bonds(T.tt_identity(bs)), lambda i: 1)
    mt = T.tt_sub(T.tt_triu_one_matrix(dim - bs), T.tt_identity(dim - bs))
    op1 = _split_diag(mt) + _placed(T.tt_split_bonds(T.tt_one_matrix(bs)), lambda i: (i + 1) % 2)
    mt = T.tt_sub(T.tt_tril_one_matrix(dim - bs), T.tt_identity(dim - bs))
    op2 = _split_diag(mt) + _placed(T.tt_split_bonds(T.tt_one_matrix(bs)), lambda i: i % 2)
    return T.tt_reshape(T.tt_rank_reduce(_q_prefix() + T.tt_sum(op0, op1, op2)), (4, 4))


def _diag_block_sum_op(bs, dim):
    op = _placed(T.tt_split_bonds(T.tt_identity(dim - bs)), lambda i: 0) + _split_diag(T.tt_identity(bs))
    op2 = _split_diag(T.tt_identity(dim - bs)) + _split_diag(T.tt_sub(T.tt_one_matrix(bs), T.tt_identity(bs)))
    return T.tt_reshape(T.tt_rank_reduce(_q_prefix() + T.tt_add(op, op2)), (4, 4))


def _h(a):
    return D.from_numpy(a)


def _eh(i, j):
    e = np.zeros((1, 2, 2, 1))
    e[:, i, j] += 1
    return e


def _Q_m_P_op(dim):
    qp = [E(0, 0), E(1, 0)]
    for _ in range(dim):
        qp.extend([_h(np.concatenate((_eh(0, 0), _eh(1, 1)), axis=-1)), _h(np.concatenate((_eh(0, 0), _eh(0, 1)), axis=0))])
    pp = [_h(-_eh(0, 0)), E(1, 1)] + _split_diag(T.to_device([_eh(0, 0) + _eh(1, 0) for _ in range(dim)]))
    p1 = T.tt_add(qp, pp)
    qp2 = [E(1, 0), E(0, 0)]
    for _ in range(dim):
        qp2.extend([_h(np.concatenate((_eh(0, 0), _eh(0, 1)), axis=-1)), _h(np.concatenate((_eh(0, 0), _eh(1, 1)), axis=0))])
    pp2 = [_h(-_eh(1, 1)), E(0, 0)] + _split_diag(T.to_device([_eh(0, 0) + _eh(0, 1) for _ in range(dim)]))
    p2 = T.tt_add(qp2, pp2)
    return T.tt_reshape(T.tt_add(p2, p1), (4, 4))


def _padding_op(dim):
    mt = [_h(_eh(0, 1) + _eh(1, 0) + _eh(1, 1))] + T.tt_one_matrix(dim)
    mt = T.tt_sub(mt, [E(0, 1)] + [_h(_eh(0, 0) + _eh(1, 0)) for _ in range(dim)])
    mt = T.tt_sub(mt, [E(1, 0)] + [_h(_eh(0, 0) + _eh(0, 1)) for _ in range(dim)])
    return T.tt_reshape(T.tt_rank_reduce(_split_diag(mt)), (4, 4))


def graphm_create_problem(n, max_rank, verbose=True):
    """`psd_system/graphm/graphm.py:150-229`"""
    if verbose:
        print("Creating Problem...")
    GA = tt_random_graph(n, max_rank, verbose=verbose)
    GB = tt_random_graph(n, max_rank, verbose=verbose)
    C = [E(0, 0)] + GB + GA
    L = _partial_trace_op(n, 2 * n)
    pJ = _partial_J_trace_op(n, 2 * n)
    pJb = [E(0, 0)] + T.tt_sub(T.tt_tril_one_matrix(n), T.tt_identity(n)) + [E(0, 1) for _ in range(n)]
    pJb = T.tt_add(pJb, [E(0, 0)] + T.tt_sub(T.tt_triu_one_matrix(n), T.tt_identity(n)) + [E(1, 0) for _ in range(n)])
    pJb = T.tt_rank_reduce(T.tt_add(pJb, [E(0, 0)] + T.tt_sub(T.tt_identity(n), [E(0, 0) for _ in range(n)])
                                    + [E(1, 1) for _ in range(n)]))
    L = T.tt_rank_reduce(T.tt_add(L, pJ), 1e-12)
    bias = pJb
    L = T.tt_rank_reduce(T.tt_add(L, _diag_block_sum_op(n, 2 * n)), 1e-12)
    bias = T.tt_rank_reduce(T.tt_add(bias, [E(0, 0) for _ in range(n + 1)] + T.tt_identity(n)))
    L = T.tt_rank_reduce(T.tt_add(L, _Q_m_P_op(2 * n)), 1e-12)
    mask = T.tt_rank_reduce([E(0, 0)] + T.tt_sub(T.tt_one_matrix(n), T.tt_identity(n))
                            + T.tt_sub(T.tt_one_matrix(n), T.tt_identity(n)))
    pad = [_h(1 - _eh(0, 0))] + T.tt_one_matrix(2 * n)
    pad = T.tt_sub(pad, [E(0, 1)] + [_h(_eh(0, 0) + _eh(1, 0)) for _ in range(2 * n)])
    pad = T.tt_sub(pad, [E(1, 0)] + [_h(_eh(0, 0) + _eh(0, 1)) for _ in range(2 * n)])
    lag_y = T.tt_sub(T.tt_one_matrix(2 * n + 1), T.tt_sum(
        pad,
        [E(0, 1)] + [_h(_eh(0, 0) + _eh(1, 0)) for _ in range(2 * n)],
        [E(1, 0)] + [_h(_eh(0, 0) + _eh(0, 1)) for _ in range(2 * n)],
        [E(0, 0)] + [E(0, 0) for _ in range(n)] + T.tt_identity(n),
        [E(0, 0)] + T.tt_identity(n) + T.tt_sub(T.tt_one_matrix(n), T.tt_identity(n)),
        pJb,
        [E(0, 0)] + T.tt_sub(T.tt_one_matrix(n), T.tt_identity(n)) + T.tt_identity(n)))
    lag_t = T.tt_sub(T.tt_one_matrix(2 * n + 1), mask)
    lag = {"y": T.tt_diag_op(lag_y), "t": T.tt_diag_op(lag_t)}
    scale = max(2 ** (2 * n + 1 - 7), 1)
    bias = T.tt_normalise(bias, radius=scale)
    L = T.tt_rank_reduce(T.tt_add(L, _padding_op(2 * n)), 1e-12)
    bias = T.tt_rank_reduce(T.tt_add(bias, [E(1, 1)] + T.tt_identity(2 * n)))
    return T.tt_normalise(C, radius=scale), L, bias, mask, lag


PROBLEMS = {"maxcut": maxcut_create_problem, "corr_clust": corr_clust_create_problem,
            "graphm": graphm_create_problem, "max_stable_set": max_stable_set_create_problem}
