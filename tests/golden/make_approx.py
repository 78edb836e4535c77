"""Golden vectors for the ALS approximate products from the REFERENCE itself (build container only):

    OPENBLAS_NUM_THREADS=1 python tests/golden/make_approx.py

Runs `tt_approx_mat_mat_mul` / `tt_approx_mat_vec_mul` (`src/tt_als.py:1502-1762`) of the
reference (imported as make_golden.py does) on seeded inputs whose rank products exceed the exact
limits (40 / 80), and writes inputs, output ranks, dense outputs and the next MT19937 draw to
`tests/golden/approx.npz`.  Only data is written."""
import os
import sys

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

import numpy as np  # noqa: E402

from make_golden import _import_reference  # noqa: E402
from make_prims import _put_tt  # noqa: E402


def cases():
    """(name, d, matrix ranks, operand ranks, operand is matrix, tol, seed)"""
    return [("mm0", 6, [1, 5, 7, 7, 7, 5, 1], [1, 5, 7, 7, 7, 5, 1], True, 1e-6, 11),
            ("mv0", 6, [1, 5, 7, 7, 7, 5, 1], [1, 4, 12, 12, 12, 4, 1], False, 1e-6, 11),
            ("mm1", 5, [1, 4, 9, 9, 4, 1], [1, 4, 8, 8, 4, 1], True, 1e-4, 3)]


def inputs(d, ra, rb, mat):
    rng = np.random.RandomState(5 + d)
    a = [rng.randn(ra[i], 2, 2, ra[i + 1]) for i in range(d)]
    b = [rng.randn(rb[i], 2, 2, rb[i + 1]) if mat else rng.randn(rb[i], 2, rb[i + 1]) for i in range(d)]
    return a, b


def dense(tt):
    t = tt[0]
    for c in tt[1:]:
        t = np.tensordot(t, c, axes=(-1, 0))
    return t


def main():
    rops, rals, _ = _import_reference(True)
    out = {}
    for name, d, ra, rb, mat, tol, seed in cases():
        a, b = inputs(d, ra, rb, mat)
        _put_tt(out, f"{name}/a", a)
        _put_tt(out, f"{name}/b", b)
        np.random.seed(seed)
        fn = rals.tt_approx_mat_mat_mul if mat else rals.tt_approx_mat_vec_mul
        res = fn([c.copy() for c in a], [c.copy() for c in b], tol=tol)
        out[f"{name}/next_randint"] = np.array(np.random.randint(0, 1 << 30))
        out[f"{name}/ranks"] = np.array(rops.tt_ranks(res))
        out[f"{name}/dense"] = dense(res)
        out[f"{name}/tol"] = np.array(tol)
        out[f"{name}/seed"] = np.array(seed)
    np.savez_compressed(os.path.join(HERE, "approx.npz"), **out)
    print("wrote", len(out), "arrays to approx.npz")


if __name__ == "__main__":
    main()
