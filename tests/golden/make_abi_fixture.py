"""Fixture for the C-ABI test (tests/c/test_abi.cpp): one local KKT system of the Schur-reduced
operator (`MatVecWrapper`, `cy_src/lgmres_cy.pyx:203-331`) from the reference's golden operator
shapes and data (prims.npz `mv2`, scaled by 0.12 with identity added to the B00 and B21 blocks so
that LGMRES converges) and a seeded right-hand side,
and the oracle's PETSc-LGMRES solution of it (oracle/petsc_lgmres.py).  Data only.

    python tests/golden/make_abi_fixture.py    ->  tests/golden/abi_lgmres.bin"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.ipm import SchurMatVec  # noqa: E402
from oracle.petsc_lgmres import lgmres  # noqa: E402

G = np.load(os.path.join(HERE, "prims.npz"))
KEYS = [(0, 0), (0, 1), (2, 1), (2, 2)]


def main(ci=2):
    L = {k: G[f"mv{ci}/L{k[0]}{k[1]}"].copy() for k in KEYS}
    A = {k: G[f"mv{ci}/A{k[0]}{k[1]}"].copy() for k in KEYS}
    R = {k: G[f"mv{ci}/R{k[0]}{k[1]}"].copy() for k in KEYS}
    invI = G[f"mv{ci}/invI"]
    # the golden operators are Gaussian (LGMRES needs > 300 iterations on them); make the two
    # diagonal-position blocks identity-dominated so the system is a well-posed local KKT system
    for k in KEYS:
        for T in (L, A, R):
            T[k] *= 0.12
    for k in [(0, 0), (2, 1)]:
        r_, n_ = L[k].shape[0], A[k].shape[1]
        L[k][:, 0, :] += np.eye(r_)
        A[k][0, :, :, 0] += np.eye(n_)
        R[k][:, 0, :] += np.eye(R[k].shape[0])
    r, n, RR = invI.shape
    s = L[0, 0].shape[1]
    m = r * n * RR
    b = np.random.default_rng(2024).standard_normal(2 * m)
    restart = min(m, 100)
    info = {}
    x = lgmres(SchurMatVec(L, A, R, invI, invI.shape).matvec, b, rtol=1e-5, max_it=300, restart=restart,
               augment=max(restart // 10, 3), info=info)
    head = np.array([r, n, RR, s, info["its"], m, restart, max(restart // 10, 3)], dtype=np.int64)
    body = np.concatenate([np.concatenate([L[k].ravel(), A[k].ravel(), R[k].ravel()]) for k in KEYS] +
                          [invI.ravel(), b, x])
    with open(os.path.join(HERE, "abi_lgmres.bin"), "wb") as f:
        f.write(head.tobytes())
        f.write(body.astype(np.float64).tobytes())
    print("abi_lgmres.bin:", head.tolist(), body.size, "doubles")


if __name__ == "__main__":
    main()
