"""Primitive-level golden vectors from the reference (called by make_golden.py, build container only).

Each case stores seeded inputs and the reference's outputs.  TT outputs are stored as ranks +
dense reconstruction (gauge-free: SVD/QR factors differ in sign/rotation between LAPACK and
the MI355X Jacobi/Householder kernels); contraction outputs are stored directly."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _rand_tt(rng, d, n, r, shape=None):
    rk = [1] + [r] * (d - 1) + [1]
    shp = shape if shape is not None else (n,)
    return [rng.standard_normal((rk[i], *shp, rk[i + 1])) for i in range(d)]


def _dense(tt):
    t = tt[0]
    for c in tt[1:]:
        t = np.tensordot(t, c, axes=(-1, 0))
    return np.sum(t, axis=(0, -1))


def _put_tt(out, key, tt):
    out[key + "/n"] = np.array(len(tt))
    for i, c in enumerate(tt):
        out[f"{key}/{i}"] = np.asarray(c)


def main(import_reference):
    rops, rals, ripm = import_reference(True)
    out = {}
    rng = np.random.default_rng(1234)
    # ---- rounding (cy_src/tt_ops_cy.pyx:179-388) on vector TTs (r,4,R) and matrix TTs (r,2,2,R)
    for ci, (d, r, shp, eps) in enumerate([(5, 3, (4,), 1e-10), (6, 5, (4,), 1e-3), (4, 4, (2, 2), 1e-6),
                                          (7, 6, (4,), 1e-12), (3, 2, (4, 4), 1e-8)]):
        tt = _rand_tt(rng, d, None, r, shp)
        # make it low-rank-ish: add a small perturbation of a rank-1 tensor
        for i in range(d):
            tt[i][..., 1:] *= 1e-4
        _put_tt(out, f"round{ci}/in", tt)
        out[f"round{ci}/eps"] = np.array(eps)
        res = rops.tt_rank_reduce([c.copy() for c in tt], eps)
        out[f"round{ci}/ranks"] = np.array(rops.tt_ranks(res))
        out[f"round{ci}/dense"] = _dense(res)
        if len(shp) == 2:  # the PSD variant adds eye(n) and needs square physical axes
            res = rops.tt_psd_rank_reduce([c.copy() for c in tt], eps)
            out[f"round{ci}/psd_ranks"] = np.array(rops.tt_ranks(res))
            out[f"round{ci}/psd_dense"] = _dense(res)
    # ---- zip-up products (cy_src/tt_ops_cy.pyx:428-502)
    for ci, (d, ra, rx, eps) in enumerate([(5, 3, 2, 1e-12), (6, 4, 3, 1e-6), (4, 2, 4, 1e-18)]):
        A = _rand_tt(rng, d, None, ra, (4, 4))
        x = _rand_tt(rng, d, None, rx, (4,))
        M1 = _rand_tt(rng, d, None, ra, (2, 2))
        M2 = _rand_tt(rng, d, None, rx, (2, 2))
        _put_tt(out, f"zip{ci}/A", A)
        _put_tt(out, f"zip{ci}/x", x)
        _put_tt(out, f"zip{ci}/M1", M1)
        _put_tt(out, f"zip{ci}/M2", M2)
        out[f"zip{ci}/eps"] = np.array(eps)
        mv = rops.tt_fast_matrix_vec_mul(A, x, eps)
        out[f"zip{ci}/mv_dense"] = _dense(mv)
        out[f"zip{ci}/mv_ranks"] = np.array(rops.tt_ranks(mv))
        mm = rops.tt_fast_mat_mat_mul(M1, M2, eps)
        out[f"zip{ci}/mm_dense"] = _dense(mm)
        out[f"zip{ci}/mm_ranks"] = np.array(rops.tt_ranks(mm))
        hd = rops.tt_fast_hadamard(M1, M2, eps)
        out[f"zip{ci}/had_dense"] = _dense(hd)
        out[f"zip{ci}/ip"] = np.array(rops.tt_inner_prod(M1, M2))
    # ---- environment updates + local apply (src/tt_als.py:190-265)
    for ci, (r, s, R, S, n) in enumerate([(3, 2, 4, 3, 4), (7, 5, 6, 4, 4), (13, 10, 13, 10, 4)]):
        P = rng.standard_normal((r, s, r))
        xl = rng.standard_normal((r, n, R))
        A = rng.standard_normal((s, n, n, S))
        Q = rng.standard_normal((R, S, R))
        v = rng.standard_normal((r, n, R))
        b = rng.standard_normal((s, n, S))
        Pb = rng.standard_normal((s, r))
        Qb = rng.standard_normal((S, R))
        for k, val in dict(P=P, xl=xl, A=A, Q=Q, v=v, b=b, Pb=Pb, Qb=Qb).items():
            out[f"env{ci}/{k}"] = val
        out[f"env{ci}/fwd"] = rals.compute_phi_fwd_A(P, xl, A, xl)
        out[f"env{ci}/bck"] = rals.compute_phi_bck_A(Q, xl, A, xl)
        out[f"env{ci}/fwd_rhs"] = rals.compute_phi_fwd_rhs(Pb, b, xl)
        out[f"env{ci}/bck_rhs"] = rals.compute_phi_bck_rhs(Qb, b, xl)
        out[f"env{ci}/apply"] = rals.cached_einsum("lsr,smnS,LSR,rnR->lmL", P, A, Q, v)
        out[f"env{ci}/apply_t"] = rals.cached_einsum("lsr,smnS,LSR,lmL->rnR", P, A, Q, v)
        out[f"env{ci}/local_rhs"] = rals.cached_einsum("br,bmB,BR->rmR", Pb, b, Qb)
    # ---- Schur-reduced KKT matvec (cy_src/lgmres_cy.pyx:203-331)
    for ci, (r, R, s) in enumerate([(2, 3, 2), (5, 4, 3), (9, 11, 6)]):
        n = 4
        keys = [(0, 0), (0, 1), (2, 1), (2, 2)]
        Ls = {k: rng.standard_normal((r, s, r)) for k in keys}
        As = {k: rng.standard_normal((s, n, n, s)) for k in keys}
        Rs = {k: rng.standard_normal((R, s, R)) for k in keys}
        invI = rng.uniform(0.5, 2.0, (r, n, R))
        x = rng.standard_normal(2 * r * n * R)
        mw = ripm.MatVecWrapper(Ls[0, 0], Ls[0, 1], Ls[2, 1], Ls[2, 2], As[0, 0], As[0, 1], As[2, 1], As[2, 2],
                                Rs[0, 0], Rs[0, 1], Rs[2, 1], Rs[2, 2], invI, r, n, R)
        for k in keys:
            out[f"mv{ci}/L{k[0]}{k[1]}"] = Ls[k]
            out[f"mv{ci}/A{k[0]}{k[1]}"] = As[k]
            out[f"mv{ci}/R{k[0]}{k[1]}"] = Rs[k]
        out[f"mv{ci}/invI"] = invI
        out[f"mv{ci}/x"] = x
        out[f"mv{ci}/y"] = np.array(mw.matvec(x), copy=True)
    # ---- normalise / scale RNG coupling (cy_src/tt_ops_cy.pyx:94-114,522-526)
    np.random.seed(7)
    tt = _rand_tt(rng, 5, None, 3, (4,))
    _put_tt(out, "norm/in", tt)
    res = rops.tt_normalise(tt, radius=np.sqrt(10))
    out["norm/dense"] = _dense(res)
    out["norm/next_randint"] = np.array(np.random.randint(0, 1 << 30))
    np.savez_compressed(os.path.join(HERE, "prims.npz"), **out)
    print("wrote", len(out), "arrays to prims.npz")
