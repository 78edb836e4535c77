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
    # ---- mask rounding (cy_src/tt_ops_cy.pyx:328-388): matrix TTs + a rank-2 0/1-ish mask TT
    for ci, (d, r, eps) in enumerate([(5, 4, 5e-4), (6, 3, 1e-3), (4, 5, 1e-10)]):
        tt = _rand_tt(rng, d, None, r, (2, 2))
        for i in range(d):
            tt[i][..., 1:] *= 1e-6
        mask = _rand_tt(rng, d, None, 2, (2, 2))
        _put_tt(out, f"mask{ci}/in", tt)
        _put_tt(out, f"mask{ci}/mask", mask)
        out[f"mask{ci}/eps"] = np.array(eps)
        res = rops.tt_mask_rank_reduce([c.copy() for c in tt], [c.copy() for c in mask], eps)
        out[f"mask{ci}/ranks"] = np.array(rops.tt_ranks(res))
        out[f"mask{ci}/dense"] = _dense(res)
    # ---- rank retraction (src/tt_ops.py:132-152) on a block TT (one (r, B, 4, R) core) and a plain TT
    for ci, (d, r, B, up) in enumerate([(5, 6, 3, 3), (6, 9, 4, 4), (4, 5, 0, 2)]):
        tt = _rand_tt(rng, d, None, r, (4,))
        if B:
            k = d // 2
            tt[k] = rng.standard_normal((tt[k].shape[0], B, 4, tt[k].shape[-1]))
        _put_tt(out, f"retract{ci}/in", tt)
        out[f"retract{ci}/upper"] = np.array([up] * (d - 1))
        res = rops.tt_rank_retraction([c.copy() for c in tt], [up] * (d - 1))
        out[f"retract{ci}/ranks"] = np.array(rops.tt_ranks(res))
        out[f"retract{ci}/dense"] = _dense(res)
    # ---- 3-block (inequality) Schur-reduced KKT matvec, fixed mode (cy_src/lgmres_cy.pyx:379-510 with
    #      :510 returning the array; the fixed module is what import_reference(True) loads)
    for ci, (r, R, s) in enumerate([(2, 3, 2), (5, 4, 3), (7, 9, 5)]):
        n = 4
        keys = [(0, 0), (0, 1), (2, 1), (2, 2), (3, 1), (3, 3)]
        Ls = {k: rng.standard_normal((r, s, r)) for k in keys}
        As = {k: rng.standard_normal((s, n, n, s)) for k in keys}
        Rs = {k: rng.standard_normal((R, s, R)) for k in keys}
        invI = rng.uniform(0.5, 2.0, (r, n, R))
        x = rng.standard_normal(3 * r * n * R)
        mw = ripm.IneqMatVecWrapper(*[Ls[k] for k in keys], *[As[k] for k in keys], *[Rs[k] for k in keys],
                                    invI, r, n, R)
        for k in keys:
            out[f"imv{ci}/L{k[0]}{k[1]}"] = Ls[k]
            out[f"imv{ci}/A{k[0]}{k[1]}"] = As[k]
            out[f"imv{ci}/R{k[0]}{k[1]}"] = Rs[k]
        out[f"imv{ci}/invI"] = invI
        out[f"imv{ci}/x"] = x
        out[f"imv{ci}/y"] = np.array(mw.matvec(x), copy=True)
    np.savez_compressed(os.path.join(HERE, "prims.npz"), **out)
    print("wrote", len(out), "arrays to prims.npz")
