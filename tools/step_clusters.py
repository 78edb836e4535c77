"""Degeneracy of the reference's step-size local eigenproblems (tests/golden/step.npz, CPU only).

    python tools/step_clusters.py [CASE ...]

For every recorded two-site local solve of `_step_size_local_solve` (`src/tt_als.py:931-1038`,
dense branch): m, the smallest eigenvalue of M = A / step + D and how many eigenvalues lie within
1e-8 * ||M|| of it (the cluster ARPACK's Krylov vector and an exact dense eigenvector may pick
different members of), and the same for the generalised pencil (-D, A) the step-limiting branch
solves.  Test infrastructure: reads only the committed fixture."""
import os
import sys

import numpy as np
import scipy.linalg as sla

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
from tests import step_cases as SC  # noqa: E402

TWO_SITE = "lsr,smnk,kptS,LSR->lmpLrntR"


def cluster(w, rel=1e-8):
    tol = rel * max(np.abs(w).max(), 1e-300)
    return int(np.sum(np.abs(w - w[0]) <= tol))


def main(cases):
    for c in cases:
        for j in range(SC.nlocal(c)):
            args, bwd, st, exp = SC.local(c, j)
            p1, p2, XAX, Ak, Akp, XAX2, XDX, Dk, Dkp, XDX2, step = args[:11]
            sh = SC.product(p1, p2).shape
            m = int(np.prod(sh))
            if sh[0] * sh[-1] > args[11]:
                print(f"{c} l{j} m={m} lobpcg branch")
                continue
            Dm = np.einsum(TWO_SITE, XDX, Dk, Dkp, XDX2, optimize=True).reshape(m, m)
            Am = np.einsum(TWO_SITE, XAX, Ak, Akp, XAX2, optimize=True).reshape(m, m)
            Dm, Am = 0.5 * (Dm + Dm.T), 0.5 * (Am + Am.T)
            w = np.linalg.eigvalsh(Am / step + Dm)
            line = f"{c} l{j} m={m} lam_min {w[0]: .3e} cluster {cluster(w)}"
            try:
                g = sla.eigh(-Dm, Am, eigvals_only=True)[::-1]
                line += f" | gen lam_max {g[0]:.6e} cluster {cluster(g)}"
            except (np.linalg.LinAlgError, ValueError):
                line += " | gen: A not positive definite"
            shapes = "" if j not in SC.DEVICE_RANK_DEPARTURES.get(c, set()) else "  <- device rank departure"
            print(line + shapes)


if __name__ == "__main__":
    main(sys.argv[1:] or SC.CASES)
