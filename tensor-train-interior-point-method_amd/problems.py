"""Problem generators -- drop-in for `psd_system/{maxcut,corr_clust,graphm,max_stable_set}/<p>.py`
`create_problem(dim, rank)` (problem creation, out of the timed region).

The generators run on the host in NumPy/LAPACK (`host_tt.py` says why: the random-graph sampler's
accept/reject test is a 1e-12 rank decision at LAPACK's rounding-noise level, so only LAPACK's
arithmetic reproduces the reference's samples and MT19937 stream), then the created TT cores
are uploaded once as fp64 device tensors.  Everything the IPM does with them runs on the device.
Each generator follows the reference module cited in its section header."""
import copy

import numpy as np

from . import dev as D
from . import host_tt as T

E = T.E


def _up(x):
    """host TT (list of ndarrays) / dict of TTs -> device tensors"""
    if isinstance(x, dict):
        return {k: _up(v) for k, v in x.items()}
    return [D.from_numpy(c) for c in x]


# ---------------------------------------------------------------- maxcut (`psd_system/maxcut/maxcut.py`)
def _diag_constraint_op(dim):
    eye = T.identity(dim)
    return T.diag_op(eye), eye


def _maxcut(dim, rank, verbose=True):
    scale = np.sqrt(dim)
    g = T.rank_reduce(T.random_graph(dim, rank, verbose=verbose))
    lap = T.sub(T.diag(T.fast_matrix_vec_mul(g, [np.ones((1, 2, 1)) for _ in range(dim)], 1e-12)), g)
    L, b = _diag_constraint_op(dim)
    lag_y = T.diag_op(T.sub(T.one_matrix(dim), T.identity(dim)))
    return (T.reshape(T.normalise(lap, radius=scale), (4,)), L,
            T.reshape(T.normalise(b, radius=scale), (4,)), lag_y)


# ---------------------------------------------------------------- corr_clust (`psd_system/corr_clust/corr_clust.py`)
def _corr_clust(dim, rank, verbose=True):
    scale = np.sqrt(dim)
    g = T.rank_reduce(T.random_graph(dim, rank, verbose=verbose), 1e-10)
    mg = T.rank_reduce(T.random_graph(dim, 1, verbose=verbose), 1e-10)
    sim = T.rank_reduce(T.fast_hadamard(g, mg, 1e-12), 1e-10)
    dis = T.rank_reduce(T.fast_hadamard(g, T.sub(T.one_matrix(dim), mg), 1e-12), 1e-10)
    lap = T.sub(T.diag(T.fast_matrix_vec_mul(dis, [np.ones((1, 2, 1)) for _ in range(dim)], 1e-12)), dis)
    obj = T.rank_reduce(T.add(sim, lap), 1e-10)
    L, b = _diag_constraint_op(dim)
    lag = {"y": T.diag_op(T.sub(T.one_matrix(dim), T.identity(dim))),
           "t": T.diag_op(T.sub(T.one_matrix(dim), g))}
    return (T.reshape(T.normalise(obj, radius=scale), (4,)), L,
            T.reshape(T.normalise(b, radius=scale), (4,)), g, lag)


# ---------------------------------------------------------------- max_stable_set
def _G_entrywise_mask_op(G):
    basis = []
    for gc in T.split_bonds(copy.deepcopy(G)):
        core = np.zeros((gc.shape[0], 2, 2, gc.shape[-1]))
        core[:, 0, 0] = gc[:, 0]
        core[:, 1, 1] = gc[:, 1]
        basis.append(core)
    return T.rank_reduce(T.reshape(basis, (4, 4)))


def _tr_constraint(dim):
    op = []
    for c in T.split_bonds([np.eye(2).reshape(1, 2, 2, 1) for _ in range(dim)]):
        core = np.zeros((c.shape[0], 2, 2, c.shape[-1]))
        core[:, 0] = c
        op.append(core)
    return T.rank_reduce(T.reshape(op, (4, 4))), [E(0, 0) for _ in range(dim)]


def _max_stable_set(dim, rank, verbose=True):
    scale = np.sqrt(dim)
    G = T.rank_reduce(T.random_graph(dim, rank, verbose=verbose))
    obj = T.one_matrix(dim)
    L, b = _tr_constraint(dim)
    L = T.rank_reduce(T.add(L, _G_entrywise_mask_op(G)))
    lag_y = T.rank_reduce(T.diag_op(T.sub(T.one_matrix(dim), T.add(G, b))))
    return (T.reshape(T.normalise(obj, radius=scale), (4,)), L,
            T.reshape(T.normalise(b, radius=scale), (4,)), lag_y)


# ---------------------------------------------------------------- graphm (`psd_system/graphm/graphm.py`)
Q_PREFIX = [np.array([[1.0, 0.0], [0.0, 0.0]]).reshape(1, 2, 2, 1),
            np.array([[1.0, 0.0], [0.0, 0.0]]).reshape(1, 2, 2, 1)]


def _partial_trace_op(bs, dim):
    op = T.diag(T.split_bonds(T.sub(T.one_matrix(dim - bs), T.identity(dim - bs))))
    blk = T.diag(T.split_bonds(T.identity(bs)))
    return T.reshape(T.rank_reduce(Q_PREFIX + op + blk), (4, 4))


def _partial_J_trace_op(bs, dim):
    mt = T.sub(T.identity(dim - bs), [E(0, 0) for _ in range(dim - bs)])
    b0 = []
    for c in T.split_bonds(T.identity(bs)):
        core = np.zeros((c.shape[0], 2, 2, c.shape[-1]))
        core[:, 1] = c
        b0.append(core)
    op0 = T.diag(T.split_bonds(mt)) + b0
    mt = T.sub(T.triu_one_matrix(dim - bs), T.identity(dim - bs))
    b1 = []
    for i, c in enumerate(T.split_bonds(T.one_matrix(bs))):
        core = np.zeros((c.shape[0], 2, 2, c.shape[-1]))
        core[:, (i + 1) % 2] = c
        b1.append(core)
    op1 = T.diag(T.split_bonds(mt)) + b1
    mt = T.sub(T.tril_one_matrix(dim - bs), T.identity(dim - bs))
    b2 = []
    for i, c in enumerate(T.split_bonds(T.one_matrix(bs))):
        core = np.zeros((c.shape[0], 2, 2, c.shape[-1]))
        core[:, i % 2] = c
        b2.append(core)
    op2 = T.diag(T.split_bonds(mt)) + b2
    return T.reshape(T.rank_reduce(Q_PREFIX + T.tt_sum(op0, op1, op2)), (4, 4))


def _diag_block_sum_op(bs, dim):
    op = []
    for c in T.split_bonds(T.identity(dim - bs)):
        core = np.zeros((c.shape[0], 2, 2, c.shape[-1]))
        core[:, 0] = c
        op.append(core)
    op = op + T.diag(T.split_bonds(T.identity(bs)))
    op2 = T.diag(T.split_bonds(T.identity(dim - bs))) + T.diag(T.split_bonds(T.sub(T.one_matrix(bs), T.identity(bs))))
    return T.reshape(T.rank_reduce(Q_PREFIX + T.add(op, op2)), (4, 4))


def _Q_m_P_op(dim):
    qp = [E(0, 0), E(1, 0)]
    for _ in range(dim):
        qp.extend([np.concatenate((E(0, 0), E(1, 1)), axis=-1), np.concatenate((E(0, 0), E(0, 1)), axis=0)])
    pp = [-E(0, 0), E(1, 1)] + T.diag(T.split_bonds([E(0, 0) + E(1, 0) for _ in range(dim)]))
    p1 = T.add(qp, pp)
    qp2 = [E(1, 0), E(0, 0)]
    for _ in range(dim):
        qp2.extend([np.concatenate((E(0, 0), E(0, 1)), axis=-1), np.concatenate((E(0, 0), E(1, 1)), axis=0)])
    pp2 = [-E(1, 1), E(0, 0)] + T.diag(T.split_bonds([E(0, 0) + E(0, 1) for _ in range(dim)]))
    p2 = T.add(qp2, pp2)
    return T.reshape(T.add(p2, p1), (4, 4))


def _padding_op(dim):
    mt = [E(0, 1) + E(1, 0) + E(1, 1)] + T.one_matrix(dim)
    mt = T.sub(mt, [E(0, 1)] + [E(0, 0) + E(1, 0) for _ in range(dim)])
    mt = T.sub(mt, [E(1, 0)] + [E(0, 0) + E(0, 1) for _ in range(dim)])
    return T.reshape(T.rank_reduce(T.diag(T.split_bonds(mt))), (4, 4))


def _graphm(n, max_rank, verbose=True):
    GA = T.random_graph(n, max_rank, verbose=verbose)
    GB = T.random_graph(n, max_rank, verbose=verbose)
    C = [E(0, 0)] + GB + GA
    L = _partial_trace_op(n, 2 * n)
    pJ = _partial_J_trace_op(n, 2 * n)
    pJb = [E(0, 0)] + T.sub(T.tril_one_matrix(n), T.identity(n)) + [E(0, 1) for _ in range(n)]
    pJb = T.add(pJb, [E(0, 0)] + T.sub(T.triu_one_matrix(n), T.identity(n)) + [E(1, 0) for _ in range(n)])
    pJb = T.rank_reduce(T.add(pJb, [E(0, 0)] + T.sub(T.identity(n), [E(0, 0) for _ in range(n)]) + [E(1, 1) for _ in range(n)]))
    L = T.rank_reduce(T.add(L, pJ), 1e-12)
    bias = pJb
    dbs = _diag_block_sum_op(n, 2 * n)
    dbs_b = [E(0, 0) for _ in range(n + 1)] + T.identity(n)
    L = T.rank_reduce(T.add(L, dbs), 1e-12)
    bias = T.rank_reduce(T.add(bias, dbs_b))
    L = T.rank_reduce(T.add(L, _Q_m_P_op(2 * n)), 1e-12)
    mask = T.rank_reduce([E(0, 0)] + T.sub(T.one_matrix(n), T.identity(n)) + T.sub(T.one_matrix(n), T.identity(n)))
    pad = [1 - E(0, 0)] + T.one_matrix(2 * n)
    pad = T.sub(pad, [E(0, 1)] + [E(0, 0) + E(1, 0) for _ in range(2 * n)])
    pad = T.sub(pad, [E(1, 0)] + [E(0, 0) + E(0, 1) for _ in range(2 * n)])
    lag_y = T.sub(T.one_matrix(2 * n + 1), T.tt_sum(
        pad,
        [E(0, 1)] + [E(0, 0) + E(1, 0) for _ in range(2 * n)],
        [E(1, 0)] + [E(0, 0) + E(0, 1) for _ in range(2 * n)],
        [E(0, 0)] + [E(0, 0) for _ in range(n)] + T.identity(n),
        [E(0, 0)] + T.identity(n) + T.sub(T.one_matrix(n), T.identity(n)),
        pJb,
        [E(0, 0)] + T.sub(T.one_matrix(n), T.identity(n)) + T.identity(n)))
    lag_t = T.sub(T.one_matrix(2 * n + 1), mask)
    lag = {"y": T.diag_op(lag_y), "t": T.diag_op(lag_t)}
    scale = max(2 ** (2 * n + 1 - 7), 1)
    bias = T.normalise(bias, radius=scale)
    L = T.rank_reduce(T.add(L, _padding_op(2 * n)), 1e-12)
    bias = T.rank_reduce(T.add(bias, [E(1, 1)] + T.identity(2 * n)))
    return T.normalise(C, radius=scale), L, bias, mask, lag


def maxcut_create_problem(dim, rank, verbose=True):
    """`psd_system/maxcut/maxcut.py:create_problem` -> (C, L, b, lag_y) on the device"""
    return tuple(_up(t) for t in _maxcut(dim, rank, verbose))


def corr_clust_create_problem(dim, rank, verbose=True):
    """`psd_system/corr_clust/corr_clust.py:create_problem` -> (C, L, b, mask, lag) on the device"""
    return tuple(_up(t) for t in _corr_clust(dim, rank, verbose))


def max_stable_set_create_problem(dim, rank, verbose=True):
    """`psd_system/max_stable_set/max_stable_set.py:create_problem` -> (C, L, b, lag_y)"""
    return tuple(_up(t) for t in _max_stable_set(dim, rank, verbose))


def graphm_create_problem(n, max_rank, verbose=True):
    """`psd_system/graphm/graphm.py:create_problem` -> (C, L, b, mask, lag) on the device"""
    return tuple(_up(t) for t in _graphm(n, max_rank, verbose))


PROBLEMS = {"maxcut": maxcut_create_problem, "corr_clust": corr_clust_create_problem,
            "graphm": graphm_create_problem, "max_stable_set": max_stable_set_create_problem}
