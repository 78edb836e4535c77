"""Numerics of the hand-written HIP kernels (libttk) against NumPy/SciPy fp64 references.
All tests need an MI355X."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ttipm_amd import dev as D
    return D


def _rng(seed=0):
    return np.random.default_rng(seed)


EQS = [
    ("lsr,lML,sMNS,rNR->LSR", [(3, 2, 3), (3, 4, 5), (2, 4, 4, 3), (3, 4, 5)]),
    ("LSR,lML,sMNS,rNR->lsr", [(5, 3, 5), (4, 2, 5), (6, 2, 2, 3), (4, 2, 5)]),
    ("lsr,smnS,LSR,rnR->lmL", [(13, 10, 13), (10, 4, 4, 10), (13, 10, 13), (13, 4, 13)]),
    ("lsr,smnS,LSR,lmL->rnR", [(7, 5, 6), (5, 4, 4, 3), (9, 3, 8), (7, 4, 9)]),
    ("lsr,smnS,LSR->lmLrnR", [(3, 2, 4), (2, 4, 4, 3), (5, 3, 2)]),
    ("lsr,smnS,LSR->lmL", [(3, 2, 4), (2, 4, 4, 3), (5, 3, 2)]),
    ("br,bmB,BR->rmR", [(4, 3), (4, 4, 6), (6, 5)]),
    ("ab,aijm,bijn->mn", [(3, 4), (3, 2, 2, 5), (4, 2, 2, 1)]),
    ("ij,rjR->rijR", [(4, 4), (3, 4, 5)]),
    ("rmnR,lijL->rlminjRL", [(1, 2, 2, 1), (3, 2, 2, 4)]),
    ("ik,kj->ij", [(70, 45), (45, 33)]),
    ("ik,kj->ij", [(1, 300), (300, 1)]),
]


@pytest.mark.parametrize("eq,shapes", EQS)
def test_einsum_matches_numpy(dev, eq, shapes):
    rng = _rng(1)
    ops = [rng.standard_normal(s) for s in shapes]
    ref = np.einsum(eq, *ops)
    got = dev.read(dev.einsum(eq, *[dev.from_numpy(o) for o in ops]))
    assert got.shape == ref.shape
    assert np.max(np.abs(got - ref)) <= 1e-13 * max(1.0, np.max(np.abs(ref)))


def test_einsum_strided_views_and_accumulate(dev):
    rng = _rng(2)
    A = rng.standard_normal((5, 4, 4, 6))
    x = rng.standard_normal((6, 4, 5))
    tA = dev.from_numpy(A).transpose(1, 2)  # (5,4,4,6) swapped axes view
    tx = dev.from_numpy(x).permute(2, 1, 0)  # (5,4,6) view
    out = dev.from_numpy(np.ones((5, 4, 5)))
    dev.einsum("smnS,rnS->smr", tA, tx, out=out, alpha=2.0, beta=-1.0)
    ref = 2.0 * np.einsum("smnS,rnS->smr", np.swapaxes(A, 1, 2), np.transpose(x, (2, 1, 0))) - 1.0
    assert np.allclose(dev.read(out), ref, rtol=1e-13, atol=1e-13)
    # accumulate into a strided slice of a larger tensor
    big = dev.zeros(5, 3, 4, 5)
    dev.einsum("smnS,rnS->smr", tA, tx, out=big[:, 1], beta=1.0)
    assert np.allclose(dev.read(big)[:, 1], ref / 2 + 0.5, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("eq", ["lsr,smnS,LSR,rnR->lmL", "lsr,smnS,LSR,lmL->rnR"])
@pytest.mark.parametrize("dims", [(3, 2, 5, 4), (13, 10, 13, 4), (28, 11, 20, 4), (1, 1, 1, 4)])
def test_fused_local_apply(dev, eq, dims):
    """The one-launch local operator apply against NumPy and against the generic GEMM plan,
    on strided operands (transposed operator view) with beta accumulation into a slice."""
    from ttipm_amd._lib import lib
    r, s, R, n = dims
    rng = _rng(r * 7 + s)
    P = rng.standard_normal((r + 1, s, r))
    Q = rng.standard_normal((R + 2, s + 1, R))
    A = rng.standard_normal((s, n, n, s + 1))
    fwd = eq.endswith("lmL")
    x = rng.standard_normal((r, n, R) if fwd else (r + 1, n, R + 2))
    ref = np.einsum(eq, P, A.transpose(0, 2, 1, 3), Q, x)
    dP, dQ, dx = dev.from_numpy(P), dev.from_numpy(Q), dev.from_numpy(x)
    dA = dev.from_numpy(A).transpose(1, 2)  # strided view
    out_full = dev.from_numpy(np.ones((2,) + ref.shape))
    dev.einsum(eq, dP, dA, dQ, dx, out=out_full[1], alpha=2.0, beta=-1.0, fused=True)
    got = dev.read(out_full)
    assert np.allclose(got[1], 2.0 * ref - 1.0, rtol=1e-12, atol=1e-12 * np.abs(ref).max())
    assert np.all(got[0] == 1.0)
    old = lib.ttk_einsum_set_fused(0)
    try:
        plain = dev.read(dev.einsum(eq, dP, dA, dQ, dx))
    finally:
        lib.ttk_einsum_set_fused(old)
    assert np.allclose(plain, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("eq,shapes", [
    ("ik,kj->ij", ((60, 2580), (2580, 40))),            # split-K: 4 tiles, long K
    ("ik,kj->ij", ((841, 15624), (15624, 31))),         # graphm_3's widest env step
    ("bik,bkj->bij", ((3, 17, 1100), (3, 1100, 9))),    # batched, ragged tiles
    ("lsr,lML,sMNS,rNR->LSR", ((40, 9, 40), (40, 4, 44), (9, 4, 4, 10), (40, 4, 44))),
])
@pytest.mark.parametrize("splitk", [1, 0])
def test_einsum_long_k(dev, eq, shapes, splitk):
    """long-K contraction steps (graphm_3 r=2 sizes) with and without the split-K path, with an
    accumulate (beta = 1) epilogue through the output offset tables"""
    from ttipm_amd._lib import lib
    rng = _rng(len(shapes[0]) * 31 + splitk)
    ops = [rng.standard_normal(sh) for sh in shapes]
    want = np.einsum(eq, *ops, optimize="greedy")
    base = rng.standard_normal(want.shape)
    old = lib.ttk_gemm_set_splitk(splitk)
    try:
        out = dev.from_numpy(base)
        dev.einsum(eq, *[dev.from_numpy(o) for o in ops], out=out, alpha=0.5, beta=1.0)
        got = dev.read(out)
    finally:
        lib.ttk_gemm_set_splitk(old)
    ref = 0.5 * want + base
    assert np.max(np.abs(got - ref)) <= 1e-12 * max(np.max(np.abs(ref)), 1.0) * np.sqrt(max(sh[-1] for sh in shapes))


def test_mfma_layout_asymmetric(dev):
    """A = I with an asymmetric B catches transposed C/D fragment maps."""
    B = np.arange(32 * 32, dtype=np.float64).reshape(32, 32)
    got = dev.read(dev.matmul(dev.from_numpy(np.eye(32)), dev.from_numpy(B)))
    assert np.array_equal(got, B)


@pytest.mark.parametrize("m,n", [(1, 1), (4, 4), (12, 3), (3, 12), (39, 52), (52, 39), (64, 7), (130, 40), (17, 1), (1, 9)])
def test_svd(dev, m, n):
    rng = _rng(m * 100 + n)
    A = rng.standard_normal((m, n))
    if min(m, n) > 3:
        A[:, 2] = A[:, 0] * 1e-9  # near rank deficiency
    U, S, Vt, s = dev.svd(dev.from_numpy(A))
    U, Vt = dev.read(U), dev.read(Vt)
    ref = np.linalg.svd(A, compute_uv=False)
    assert np.allclose(s, ref, rtol=1e-12, atol=1e-14 * ref[0])
    assert np.all(np.diff(s) <= 0)
    assert np.allclose((U * s) @ Vt, A, atol=1e-13 * np.abs(A).max())
    k = min(m, n)
    assert np.allclose(U.T @ U, np.eye(k), atol=1e-12)
    assert np.allclose(Vt @ Vt.T, np.eye(k), atol=1e-12)


def _check_svd(dev, A, rtol=1e-12):
    m, n = A.shape
    U, S, Vt, s = dev.svd(dev.from_numpy(A))
    U, Vt = dev.read(U), dev.read(Vt)
    ref = np.linalg.svd(A, compute_uv=False)
    assert np.allclose(s, ref, rtol=rtol, atol=1e-14 * ref[0])
    assert np.all(np.diff(s) <= 0)
    assert np.allclose((U * s) @ Vt, A, atol=1e-13 * np.abs(A).max() * max(1, np.sqrt(min(m, n)) / 4))
    k = min(m, n)
    assert np.allclose(U.T @ U, np.eye(k), atol=1e-12)
    assert np.allclose(Vt @ Vt.T, np.eye(k), atol=1e-12)


@pytest.mark.parametrize("m,n", [(5, 4), (39, 52), (52, 39), (3, 1), (1, 3)])
def test_svd_multi_workgroup_forced(dev, m, n):
    from ttipm_amd._lib import lib
    rng = _rng(m + 3 * n)
    A = rng.standard_normal((m, n))
    old = lib.ttk_svd_set_big_threshold(1)
    try:
        _check_svd(dev, A)
    finally:
        lib.ttk_svd_set_big_threshold(old)


@pytest.mark.parametrize("m,n", [(70, 40), (40, 70), (33, 33), (130, 64), (5, 3), (3, 5)])
def test_qr_blocked_forced(dev, m, n):
    from ttipm_amd._lib import lib
    rng = _rng(m * 7 + n)
    A = rng.standard_normal((m, n))
    old = lib.ttk_qr_set_big_threshold(1)
    try:
        Q, R = dev.qr(dev.from_numpy(A))
    finally:
        lib.ttk_qr_set_big_threshold(old)
    Q, R = dev.read(Q), dev.read(R)
    Qr, Rr = np.linalg.qr(A)
    k = min(m, n)
    assert np.allclose(Q @ R, A, atol=1e-13 * np.abs(A).max() * np.sqrt(k))
    assert np.allclose(Q.T @ Q, np.eye(k), atol=1e-13)
    assert np.allclose(np.tril(R, -1), 0)
    # LAPACK sign convention (beta = -sign(alpha)||x||) -> same factors as numpy/LAPACK
    assert np.allclose(R, Rr, atol=1e-11 * np.abs(A).max())


@pytest.mark.parametrize("m,n", [(1400, 256), (256, 900), (700, 500)])
def test_qr_large(dev, m, n):
    rng = _rng(m + n)
    A = rng.standard_normal((m, n))
    Q, R = dev.qr(dev.from_numpy(A))
    Q, R = dev.read(Q), dev.read(R)
    k = min(m, n)
    assert np.allclose(Q @ R, A, atol=1e-12 * np.abs(A).max() * np.sqrt(k))
    assert np.allclose(Q.T @ Q, np.eye(k), atol=1e-12)


@pytest.mark.parametrize("m,n,r", [(300, 420, 300), (520, 260, 60), (868, 1024, 217), (1400, 256, 256)])
def test_svd_large_rank_deficient(dev, m, n, r):
    """Sizes and rank structure of the 1e-12 roundings at the end of a solve."""
    rng = _rng(m + n)
    A = rng.standard_normal((m, r)) @ (rng.standard_normal((r, n)) * np.logspace(0, -13, r)[:, None])
    _check_svd(dev, A)


@pytest.mark.parametrize("case", ["graded", "clustered"])
def test_svd_large_deflated(dev, case):
    """Deflated large SVD: singular values above the deflation level are exact, the deflated
    ones are zero, and the kept triplets reconstruct A to the dropped energy."""
    rng = _rng(5)
    m, n, r = 500, 700, 240
    if case == "graded":
        s = np.logspace(0, -15, r)
    else:
        s = np.concatenate([np.full(40, np.sqrt(2.0)), np.logspace(-1, -15, r - 40)])
    Ql, _ = np.linalg.qr(rng.standard_normal((m, r)))
    Qr, _ = np.linalg.qr(rng.standard_normal((n, r)))
    A = (Ql * s) @ Qr.T
    defl = 1e-3 * 1e-12
    U, S, Vt, sv = dev.svd(dev.from_numpy(A), defl=defl)
    U, Vt = dev.read(U), dev.read(Vt)
    ref = np.linalg.svd(A, compute_uv=False)
    assert np.all(np.diff(sv) <= 0)
    k = int(np.sum(sv > 0))
    assert np.sum(ref[k:] ** 2) <= defl ** 2 * 1.01 + 1e-30
    assert np.allclose(sv[:k], ref[:k], rtol=0, atol=5e-14 * ref[0])
    assert np.abs((U[:, :k] * sv[:k]) @ Vt[:k] - A).max() <= 1e-13 * np.abs(A).max() + defl
    assert np.allclose(U[:, :k].T @ U[:, :k], np.eye(k), atol=1e-12)


def test_svd_zero_and_rank_one(dev):
    U, S, Vt, s = dev.svd(dev.zeros(6, 4))
    assert np.all(s == 0)
    U = dev.read(U)
    assert np.allclose(U.T @ U, np.eye(4), atol=1e-12)
    a = np.outer(np.arange(1, 7.0), np.arange(1, 5.0))
    U, S, Vt, s = dev.svd(dev.from_numpy(a))
    assert np.allclose(s[0], np.linalg.norm(a)) and np.all(np.abs(s[1:]) < 1e-12)


@pytest.mark.parametrize("m,n", [(4, 4), (13, 4), (4, 13), (60, 20), (200, 30), (1, 5), (5, 1)])
def test_qr_and_rq(dev, m, n):
    rng = _rng(7 + m + n)
    A = rng.standard_normal((m, n))
    Q, R = dev.qr(dev.from_numpy(A))
    Q, R = dev.read(Q), dev.read(R)
    k = min(m, n)
    assert np.allclose(Q @ R, A, atol=1e-13 * np.abs(A).max())
    assert np.allclose(Q.T @ Q, np.eye(k), atol=1e-13)
    assert np.allclose(np.tril(R, -1), 0)
    Rr, Qr = dev.rq(dev.from_numpy(A))
    Rr, Qr = dev.read(Rr), dev.read(Qr)
    assert np.allclose(Rr @ Qr, A, atol=1e-12 * np.abs(A).max())
    assert np.allclose(Qr @ Qr.T, np.eye(k), atol=1e-12)


@pytest.mark.parametrize("n,nrhs", [(1, 7), (5, 7), (40, 7), (130, 7), (200, 300), (333, 45), (700, 700)])
@pytest.mark.parametrize("blocked", [None, 1])  # default dispatch / blocked kernels forced at every n
def test_cholesky_trsm(dev, n, nrhs, blocked):
    from ttipm_amd._lib import lib
    old = lib.ttk_dense_set_block_min(blocked) if blocked else None
    try:
        rng = _rng(n)
        M = rng.standard_normal((n, n))
        A = M @ M.T + n * np.eye(n)
        L = dev.from_numpy(A)
        dev.cholesky_(L)
        Lh = dev.read(L)
        assert np.allclose(Lh, np.linalg.cholesky(A), rtol=1e-12, atol=1e-12)
        B = rng.standard_normal((n, nrhs))
        X = dev.from_numpy(B)
        dev.trsm_(L, X)
        assert np.allclose(Lh @ dev.read(X), B, atol=1e-10)
        X2 = dev.from_numpy(B)
        dev.trsm_(L, X2, trans=True)
        assert np.allclose(Lh.T @ dev.read(X2), B, atol=1e-10)
    finally:
        if old is not None:
            lib.ttk_dense_set_block_min(old)


@pytest.mark.parametrize("n,bad", [(2, 1), (150, 1), (150, 77), (300, 299)])
def test_cholesky_not_pd_raises(dev, n, bad):
    """LAPACK info semantics: the first non-positive leading minor (1-based) is reported"""
    rng = _rng(n + bad)
    M = rng.standard_normal((n, n))
    A = M @ M.T + n * np.eye(n)
    A[bad, bad] = -1e3 * n  # leading minor bad+1 is indefinite
    L = dev.from_numpy(A)
    with pytest.raises(dev.LinAlgError, match=f"{bad + 1}-th leading minor"):
        dev.cholesky_(L)


@pytest.mark.parametrize("n", [1, 6, 50, 95, 96, 200, 700, 1500])
def test_lu_solve_rcond(dev, n):
    rng = _rng(3 * n)
    A = rng.standard_normal((n, n)) + 0.1 * np.eye(n)
    b = rng.standard_normal((n, 3))
    LU = dev.from_numpy(A)
    piv = dev.lu_(LU)
    X = dev.from_numpy(b)
    dev.lu_solve_(LU, piv, X)
    assert np.allclose(A @ dev.read(X), b, atol=1e-8 * np.linalg.cond(A))


@pytest.mark.parametrize("n", [50, 96, 333, 1200])
def test_lu_matches_lapack(dev, n):
    """pivots, factors and the rcond estimate against LAPACK dgetrf / dgecon (blocked path from n=96)"""
    import ctypes
    import scipy.linalg as sla
    from ttipm_amd._lib import lib
    rng = _rng(17 * n)
    A = rng.standard_normal((n, n))
    lu_ref, piv_ref = sla.lu_factor(A)
    LU = dev.from_numpy(A)
    piv = dev.torch.empty(n, dtype=dev.torch.int32, device=dev.DEV)
    work = dev.empty(2 * n + 16)
    rc = ctypes.c_double(0.0)
    assert lib.ttk_lu_sync(dev._stream(), LU.data_ptr(), n, piv.data_ptr(), work.data_ptr(), ctypes.byref(rc)) == 0
    assert np.array_equal(piv.cpu().numpy(), piv_ref)
    assert np.abs(dev.read(LU) - lu_ref).max() <= 1e-10 * np.abs(lu_ref).max()
    anorm = np.abs(A).sum(axis=0).max()
    rcond_ref, info = sla.lapack.dgecon(lu_ref, anorm, norm="1")
    # dgecon's estimate, or -- when the comparison-matrix bound already settles the LinAlgWarning test
    # -- a certified lower bound of it that is >= 1e-13 (include/ttk.h ttk_lu_sync)
    assert 0.3 * rcond_ref <= rc.value <= 3.0 * rcond_ref or 1e-13 <= rc.value <= rcond_ref * (1 + 1e-8), \
        (rc.value, rcond_ref)
    B = rng.standard_normal((n, 2))
    X = dev.from_numpy(B)
    dev.lu_solve_(LU, piv, X)
    assert np.allclose(dev.read(X), sla.lu_solve((lu_ref, piv_ref), B), rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("n,scale", [(64, 1e-3), (300, 1e-9), (700, 1e-14), (1200, 1.0)])
def test_lu_rcond_warning_decision_matches_lapack(dev, n, scale):
    """the LinAlgWarning decision (rcond < eps) from ttk_lu_sync equals LAPACK dgecon's on matrices
    from well- to ill-conditioned (a rank-deficient part scaled by `scale`), certified bound or not"""
    import ctypes
    import scipy.linalg as sla
    from ttipm_amd._lib import lib
    rng = _rng(n)
    U, _ = np.linalg.qr(rng.standard_normal((n, n)))
    V, _ = np.linalg.qr(rng.standard_normal((n, n)))
    sv = np.ones(n)
    sv[n // 2:] = scale
    A = (U * sv) @ V.T
    lu_ref, _ = sla.lu_factor(A)
    rcond_ref, _ = sla.lapack.dgecon(lu_ref, np.abs(A).sum(axis=0).max(), norm="1")
    LU = dev.from_numpy(A)
    piv = dev.torch.empty(n, dtype=dev.torch.int32, device=dev.DEV)
    work = dev.empty(2 * n + 16)
    rc = ctypes.c_double(0.0)
    assert lib.ttk_lu_sync(dev._stream(), LU.data_ptr(), n, piv.data_ptr(), work.data_ptr(), ctypes.byref(rc)) == 0
    eps = np.finfo(float).eps
    assert (rc.value < eps) == (rcond_ref < eps), (rc.value, rcond_ref)


def test_lu_ill_conditioned_raises_warning(dev):
    A = np.array([[1.0, 1.0], [1.0, 1.0 + 1e-17]])
    A[1, 1] = 1.0 + 2 ** -52
    with pytest.raises((dev.LinAlgWarning, dev.LinAlgError)):
        dev.lu_(dev.from_numpy(A))


@pytest.mark.parametrize("n", [1, 2, 9, 64, 150])
def test_syev(dev, n):
    rng = _rng(11 * n)
    M = rng.standard_normal((n, n))
    A = M + M.T
    ev, W, evh = dev.syev(dev.from_numpy(A))
    W = dev.read(W)
    assert np.allclose(evh, np.linalg.eigvalsh(A), atol=1e-12 * max(1, np.abs(evh).max()))
    assert np.allclose(A @ W, W * evh, atol=1e-11 * max(1, np.abs(evh).max()))


def _sym_cases(n, rng):
    M = rng.standard_normal((n, n))
    yield "gauss", M + M.T
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    d = np.sort(rng.standard_normal(n))
    if n > 2:
        d[:2] = d[0]  # degenerate extreme eigenvalue
        d[-2:] = d[-1]
    yield "degenerate", (Q * d) @ Q.T
    B = rng.standard_normal((n, max(1, n // 3)))
    yield "psd_rank_deficient", B @ B.T
    yield "scaled", 1e-6 * (M + M.T) + np.diag(np.arange(n, dtype=float))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 10, 64, 100, 127, 128, 129, 139, 140, 288, 600, 800])
@pytest.mark.parametrize("largest", [False, True])
def test_syev_extreme(dev, n, largest):
    rng = _rng(7 * n + largest)
    for name, A in _sym_cases(n, rng):
        lam, v = dev.syev_extreme(dev.from_numpy(A), largest=largest)
        v = dev.read(v)
        w = np.linalg.eigvalsh(A)
        ref = w[-1] if largest else w[0]
        scale = max(1.0, np.abs(w).max())
        assert abs(lam - ref) <= 1e-12 * scale, (name, lam, ref)
        assert abs(np.linalg.norm(v) - 1.0) < 1e-12, name
        assert np.linalg.norm(A @ v - lam * v) <= 1e-10 * scale, name


@pytest.mark.parametrize("n", [5, 40, 100, 128])
def test_syev_small_matches_general_kernel(dev, n):
    """the 4-wave small-n kernel and the general one-workgroup kernel give the same eigenpair"""
    from ttipm_amd._lib import lib
    rng = _rng(11 * n)
    for name, A in _sym_cases(n, rng):
        w = np.linalg.eigvalsh(A)
        for largest in (False, True):
            gap = (w[-1] - w[-2]) if largest else (w[1] - w[0])
            if gap <= 1e-8 * max(1.0, np.abs(w).max()):
                continue  # the eigenvector of a multiple eigenvalue is not unique
            l1, v1 = dev.syev_extreme(dev.from_numpy(A), largest=largest)
            old = lib.ttk_syev_set_small(0)
            try:
                l2, v2 = dev.syev_extreme(dev.from_numpy(A), largest=largest)
            finally:
                lib.ttk_syev_set_small(old)
            v1, v2 = dev.read(v1), dev.read(v2)
            scale = max(1.0, np.abs(A).max())
            assert abs(l1 - l2) <= 1e-13 * scale * n, (name, l1, l2)
            assert min(np.abs(v1 - v2).max(), np.abs(v1 + v2).max()) <= 1e-8, name


@pytest.mark.parametrize("n", [150, 301])
def test_syev_fused_matches_two_launch(dev, n):
    """the one-launch-per-step and the two-launch multi-workgroup tridiagonalisations agree"""
    from ttipm_amd._lib import lib
    rng = _rng(13 * n)
    for name, A in _sym_cases(n, rng):
        w = np.linalg.eigvalsh(A)
        for largest in (False, True):
            gap = (w[-1] - w[-2]) if largest else (w[1] - w[0])
            if gap <= 1e-8 * max(1.0, np.abs(w).max()):
                continue
            l1, v1 = dev.syev_extreme(dev.from_numpy(A), largest=largest)
            old = lib.ttk_syev_set_fused_max(0)
            try:
                l2, v2 = dev.syev_extreme(dev.from_numpy(A), largest=largest)
            finally:
                lib.ttk_syev_set_fused_max(old)
            v1, v2 = dev.read(v1), dev.read(v2)
            scale = max(1.0, np.abs(A).max())
            assert abs(l1 - l2) <= 1e-13 * scale * n, (name, l1, l2)
            assert min(np.abs(v1 - v2).max(), np.abs(v1 + v2).max()) <= 1e-8, name


@pytest.mark.parametrize("n", [129, 150, 257, 258, 300, 513])
def test_syev_tri_one_workgroup_bit_identical(dev, n):
    """the one-workgroup tridiagonalisation (TTK_KNOB_TRI_ONE, one launch) and one launch per
    Householder step give the same eigenpair bit for bit, on every case of _sym_cases (degenerate and
    rank-deficient ones included), and the pair is an eigenpair (1e-10 residual)"""
    from ttipm_amd import _lib
    rng = _rng(17 * n)
    for name, A in _sym_cases(n, rng):
        for largest in (False, True):
            out = []
            for v in (513, 0):
                old = _set_knob(_lib.KNOB_TRI_ONE, v)
                try:
                    lam, vec = dev.syev_extreme(dev.from_numpy(A), largest=largest)
                finally:
                    _set_knob(_lib.KNOB_TRI_ONE, old)
                out.append((lam, dev.read(vec)))
            (l1, v1), (l2, v2) = out
            assert l1 == l2 and np.array_equal(v1, v2), (name, largest, l1, l2)
            scale = max(1.0, np.abs(A).max())
            assert np.linalg.norm(A @ v1 - l1 * v1) <= 1e-10 * scale * np.sqrt(n), name


@pytest.mark.parametrize("n", [3, 8, 17, 32, 40, 63])
def test_syev_small_eight_waves_bit_identical(dev, n):
    """the small extreme-eigenpair kernel with 8 waves (TTK_KNOB_SYEV_WAVES8: the same symv, the rank-2
    rows over 7 waves) and with 4 give the same eigenpair bit for bit on every case of _sym_cases"""
    from ttipm_amd import _lib
    rng = _rng(41 * n)
    for name, A in _sym_cases(n, rng):
        for largest in (False, True):
            out = []
            for v in (1, 0):
                old = _set_knob(_lib.KNOB_SYEV_WAVES8, v)
                try:
                    lam, vec = dev.syev_extreme(dev.from_numpy(A), largest=largest)
                finally:
                    _set_knob(_lib.KNOB_SYEV_WAVES8, old)
                out.append((lam, dev.read(vec)))
            (l1, v1), (l2, v2) = out
            assert l1 == l2 and np.array_equal(v1, v2), (name, largest, l1, l2)
            scale = max(1.0, np.abs(A).max())
            assert np.linalg.norm(A @ v1 - l1 * v1) <= 1e-10 * scale * np.sqrt(n), name


@pytest.mark.parametrize("n", [129, 150, 256, 300, 448, 513])
def test_syev_staged_back_transform_bit_identical(dev, n):
    """the multi-launch extreme eigenpair's back-transform with its reflectors staged through LDS
    (TTK_KNOB_BT_STAGE) and loaded from global memory one ahead give the same eigenpair bit for bit"""
    from ttipm_amd import _lib
    rng = _rng(43 * n)
    for name, A in _sym_cases(n, rng):
        for largest in (False, True):
            out = []
            for v in (1, 0):
                old = _set_knob(_lib.KNOB_BT_STAGE, v)
                try:
                    lam, vec = dev.syev_extreme(dev.from_numpy(A), largest=largest)
                finally:
                    _set_knob(_lib.KNOB_BT_STAGE, old)
                out.append((lam, dev.read(vec)))
            (l1, v1), (l2, v2) = out
            assert l1 == l2 and np.array_equal(v1, v2), (name, largest, l1, l2)
            scale = max(1.0, np.abs(A).max())
            assert np.linalg.norm(A @ v1 - l1 * v1) <= 1e-10 * scale * np.sqrt(n), name


@pytest.mark.parametrize("n", [129, 150, 256, 257, 300, 512])
def test_syev_tri_persistent_launch_bit_identical(dev, n):
    """the multi-workgroup tridiagonalisation with every Householder step in one launch
    (TTK_KNOB_TRI_PERSIST: resident workgroups, steps handed over through the arrival counter) and
    with one launch per step give the same eigenpair bit for bit on every case of _sym_cases; no
    hand-off wait timed out"""
    from ttipm_amd import _lib
    rng = _rng(31 * n)
    for name, A in _sym_cases(n, rng):
        for largest in (False, True):
            out = []
            for v in (1, 0):
                old = _set_knob(_lib.KNOB_TRI_PERSIST, v)
                try:
                    lam, vec = dev.syev_extreme(dev.from_numpy(A), largest=largest)
                finally:
                    _set_knob(_lib.KNOB_TRI_PERSIST, old)
                out.append((lam, dev.read(vec)))
            (l1, v1), (l2, v2) = out
            assert l1 == l2 and np.array_equal(v1, v2), (name, largest, l1, l2)
            scale = max(1.0, np.abs(A).max())
            assert np.linalg.norm(A @ v1 - l1 * v1) <= 1e-10 * scale * np.sqrt(n), name
    dev.check_handoffs()


@pytest.mark.parametrize("m,n,graded", [(150, 120, 0), (120, 150, 1), (300, 200, 1), (97, 97, 0), (400, 130, 0),
                                        (260, 255, 1)])
def test_svd_sweep_one_launch_bit_identical(dev, m, n, graded):
    """the multi-workgroup Jacobi SVD (min(m,n) > 96) with one launch per sweep (TTK_KNOB_SVD_SWEEP_ONE:
    resident pair waves, per-column round hand-offs) and with one launch per round give the same U, S,
    Vt bit for bit, and the factorisation holds; no hand-off wait timed out"""
    from ttipm_amd import _lib
    rng = _rng(7 * m + n)
    k = min(m, n)
    A = rng.standard_normal((m, n))
    if graded:
        Uq, _ = np.linalg.qr(rng.standard_normal((m, k)))
        Vq, _ = np.linalg.qr(rng.standard_normal((n, k)))
        A = (Uq * np.logspace(0, -15, k)) @ Vq.T
    out = []
    for v in (1, 0):
        old = _set_knob(_lib.KNOB_SVD_SWEEP_ONE, v)
        try:
            U, S, Vt, s = dev.svd(dev.from_numpy(A))
        finally:
            _set_knob(_lib.KNOB_SVD_SWEEP_ONE, old)
        out.append((dev.read(U), dev.read(S), dev.read(Vt)))
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    U, S, Vt = out[0]
    assert np.abs((U * S) @ Vt - A).max() <= 1e-12 * max(1.0, np.abs(A).max()) * np.sqrt(k)
    dev.check_handoffs()


@pytest.mark.parametrize("m,n", [(16, 4), (4, 16), (32, 32), (96, 40), (200, 97), (130, 300)])
def test_svd_tol_read_equals_svd_then_read(dev, m, n):
    """ttk_svd_tol_read (the one-workgroup SVD kernel storing S into host-coherent memory itself; the
    multi-workgroup path for min(m,n) > 96 reading S afterwards) = ttk_svd_tol + ttk_read_sync, bit
    for bit: U, S, Vt on the device and the host copy of S"""
    rng = _rng(11 * m + n)
    A = dev.from_numpy(rng.standard_normal((m, n)) * np.logspace(0, -8, n))
    old = dev._SVD_READ
    out = []
    try:
        for v in (True, False):
            dev._SVD_READ = v
            U, S, Vt, s = dev.svd(A, defl=1e-10)
            out.append((dev.read(U), dev.read(S), dev.read(Vt), s))
    finally:
        dev._SVD_READ = old
    for a, b in zip(*out):
        assert a.shape == b.shape and np.array_equal(a, b)
    assert np.array_equal(out[0][3], out[0][1])


def test_elementwise_and_reductions(dev):
    rng = _rng(5)
    a = rng.standard_normal((3, 4, 5))
    b = rng.standard_normal((3, 4, 5))
    ta, tb = dev.from_numpy(a), dev.from_numpy(b)
    assert np.isclose(dev.dot(ta, tb), np.sum(a * b), rtol=1e-13)
    assert np.isclose(dev.dot(ta.transpose(0, 2), tb.transpose(0, 2)), np.sum(a * b), rtol=1e-13)
    out = dev.zeros(3, 5, 4)
    dev.copy_(out, ta.transpose(1, 2), 2.0)
    assert np.allclose(dev.read(out), 2 * np.swapaxes(a, 1, 2))
    dev.mul_(out, ta.transpose(1, 2), tb.transpose(1, 2), 1.0, 1.0)
    assert np.allclose(dev.read(out), 2 * np.swapaxes(a, 1, 2) + np.swapaxes(a * b, 1, 2))
    r = dev.recip(dev.from_numpy(np.array([2.0, 4.0])))
    assert np.allclose(dev.read(r), [0.5, 0.25])


def test_einsum_batch_is_bit_identical(dev):
    """recorded + grouped launches (ttk_einsum_batch_*) give the same bits as one call at a time:
    environment updates (fused and pairwise), accumulation into one output, dependent chains"""
    import ctypes
    from ttipm_amd._lib import lib
    from ttipm_amd.tt_als import compute_phi_bck_A, compute_phi_fwd_A
    rng = _rng(11)
    ops = []
    for (r, s, R) in [(3, 2, 4), (7, 5, 6), (13, 10, 13), (5, 3, 5)]:
        ops.append(dict(P=dev.from_numpy(rng.standard_normal((r, s, r))),
                        Q=dev.from_numpy(rng.standard_normal((R, s, R))),
                        xl=dev.from_numpy(rng.standard_normal((r, 4, R))),
                        A=dev.from_numpy(rng.standard_normal((s, 4, 4, s))),
                        v=dev.from_numpy(rng.standard_normal((r, 4, R)))))
    big = [dev.from_numpy(rng.standard_normal((70, 45))), dev.from_numpy(rng.standard_normal((45, 33)))]

    def work():
        outs = []
        for o in ops:
            outs.append(compute_phi_fwd_A(o["P"], o["xl"], o["A"], o["xl"]))
            outs.append(compute_phi_bck_A(o["Q"], o["xl"], o["A"], o["xl"]))
            acc = dev.zeros(*o["v"].shape)
            dev.einsum("lsr,smnS,LSR,rnR->lmL", o["P"], o["A"], o["Q"], o["v"], out=acc, beta=1.0)
            dev.einsum("lsr,smnS,LSR,rnR->lmL", o["P"], o["A"], o["Q"], o["v"], out=acc, alpha=-0.5, beta=1.0)
            outs.append(acc)
            t = dev.einsum("ik,kj->ij", big[0], big[1])
            outs.append(dev.einsum("ij,kj->ik", t, big[1]))  # depends on t inside the batch
        return [dev.read(x) for x in outs]

    ref = work()
    st0 = (ctypes.c_longlong * 3)()
    lib.ttk_einsum_batch_stats(st0)
    l0 = lib.ttk_launch_count()
    outs = []  # recorded without reads inside the block (a read would flush it early)
    with dev.einsum_batch():
        for o in ops:
            outs.append(compute_phi_fwd_A(o["P"], o["xl"], o["A"], o["xl"]))
            outs.append(compute_phi_bck_A(o["Q"], o["xl"], o["A"], o["xl"]))
            acc = dev.zeros(*o["v"].shape)
            dev.einsum("lsr,smnS,LSR,rnR->lmL", o["P"], o["A"], o["Q"], o["v"], out=acc, beta=1.0)
            dev.einsum("lsr,smnS,LSR,rnR->lmL", o["P"], o["A"], o["Q"], o["v"], out=acc, alpha=-0.5, beta=1.0)
            outs.append(acc)
            t = dev.einsum("ik,kj->ij", big[0], big[1])
            outs.append(dev.einsum("ij,kj->ik", t, big[1]))
    launches = lib.ttk_launch_count() - l0
    st1 = (ctypes.c_longlong * 3)()
    lib.ttk_einsum_batch_stats(st1)
    assert st1[1] > st0[1]  # steps were recorded
    got = [dev.read(x) for x in outs]
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
    assert launches < 4 * len(ops) * 3  # grouped: far fewer launches than steps


def test_rank_scan_matches_sequential_updates(dev):
    """ttk_rank_scan_sync == the loop of copy_(res, neg, -1, 1) + dot(res, res), bit for bit"""
    rng = _rng(12)
    res0 = rng.standard_normal((5, 3, 4, 6))
    negs = rng.standard_normal((7, 5, 3, 4, 6)) * 1e-3
    r1 = dev.from_numpy(res0)
    ss_ref = []
    for q in range(7):
        dev.copy_(r1, dev.from_numpy(negs[q]), -1.0, 1.0)
        ss_ref.append(dev.dot(r1, r1))
    r2 = dev.from_numpy(res0)
    ss = dev.rank_scan(r2, dev.from_numpy(negs))
    assert list(ss) == ss_ref
    assert np.array_equal(dev.read(r1), dev.read(r2))


@pytest.mark.parametrize("eq", ["lsr,smnS,LSR,rnR->lmL", "lsr,smnS,LSR,lmL->rnR"])
@pytest.mark.parametrize("shapes", [[(44, 10, 44), (10, 4, 4, 10), (44, 10, 44), (44, 4, 44)],
                                    [(30, 18, 25), (18, 4, 4, 9), (28, 9, 33), (25, 4, 33)]])
def test_fused_apply_mfma_matches_numpy(dev, eq, shapes):
    """graphm-sized local applies (beyond the VALU kernel's FLOP range) on the MFMA stages, with and
    without accumulation, against NumPy (fp64; MFMA accumulation order -> 1e-13 relative)"""
    from ttipm_amd._lib import lib
    rng = _rng(13)
    P, A, Q = (rng.standard_normal(s) for s in shapes[:3])
    if eq.endswith("->lmL"):
        x = rng.standard_normal(shapes[3])
    else:
        x = rng.standard_normal((P.shape[0], A.shape[1], Q.shape[0]))
    ref = np.einsum(eq, P, A, Q, x)
    old = lib.ttk_fused_set_mfma(1)
    try:
        got = dev.read(dev.einsum(eq, *[dev.from_numpy(o) for o in (P, A, Q, x)], fused=True))
        out = dev.from_numpy(np.ones(ref.shape))
        dev.einsum(eq, *[dev.from_numpy(o) for o in (P, A, Q, x)], out=out, alpha=0.5, beta=2.0, fused=True)
    finally:
        lib.ttk_fused_set_mfma(old)
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(got - ref)) <= 1e-13 * scale
    assert np.max(np.abs(dev.read(out) - (0.5 * ref + 2.0))) <= 1e-13 * scale


@pytest.mark.gpu
@pytest.mark.parametrize("backward,shapes", [
    (True, [(64, 3, 64), (78, 4, 64), (4, 4, 4, 3), (78, 4, 64)]),   # nc * nd = 78 * 64 > one Q chunk
    (False, [(47, 5, 47), (47, 4, 97), (5, 4, 4, 4), (47, 4, 97)]),
    (False, [(2, 12, 97), (2, 4, 2), (12, 4, 4, 13), (97, 4, 50)]),
    (True, [(44, 10, 44), (44, 4, 44), (10, 4, 4, 10), (44, 4, 44)]),
])
def test_env_update_mfma_matches_numpy(dev, backward, shapes):
    """Environment updates of one core step (ttk_env_update: relabelled strided local applies) on the
    MFMA stages and on the default plan, against NumPy `compute_phi_*_A` (src/tt_als.py:252-257)"""
    from ttipm_amd import tt_als
    from ttipm_amd._lib import lib
    rng = _rng(17)
    P, x, A, y = (rng.standard_normal(s) for s in shapes)
    eq = "LSR,lML,sMNS,rNR->lsr" if backward else "lsr,lML,sMNS,rNR->LSR"
    ref = np.einsum(eq, P, x, A, y)
    items = [tuple(dev.from_numpy(o) for o in (P, x, A, y))]
    for mode in (1, 0):
        old = lib.ttk_fused_set_mfma(mode)
        try:
            got = dev.read(tt_als.env_update_many(backward, items)[0])
        finally:
            lib.ttk_fused_set_mfma(old)
        assert np.max(np.abs(got - ref)) <= 1e-12 * np.max(np.abs(ref)), mode


def _set_csplit(on):
    import ctypes
    from ttipm_amd import _lib
    old = ctypes.c_int(0)
    assert _lib.lib.ttk_ctx_set_knob(None, _lib.KNOB_MFMA_CSPLIT, int(on), ctypes.byref(old)) == 0
    return old.value


@pytest.mark.gpu
@pytest.mark.parametrize("eq", ["lsr,smnS,LSR,rnR->lmL", "lsr,smnS,LSR,lmL->rnR"])
@pytest.mark.parametrize("shapes", [[(14, 10, 14), (10, 4, 4, 9), (96, 9, 96), (14, 4, 96)],
                                    [(20, 10, 20), (10, 4, 4, 9), (113, 9, 113), (20, 4, 113)],
                                    [(44, 10, 44), (10, 4, 4, 10), (44, 10, 44), (44, 4, 44)]])
def test_mfma_rows_split_over_workgroups_bit_identical(dev, eq, shapes):
    """MFMA-stage apply rows with their stage-3 output tiles spread over several workgroups per row
    (TTK_KNOB_MFMA_CSPLIT) give the single-workgroup rows' results bit for bit, as one launch and
    inside an einsum batch (grouped launch), and agree with NumPy"""
    from ttipm_amd._lib import lib
    rng = _rng(31)
    P, A, Q = (rng.standard_normal(s) for s in shapes[:3])
    x = rng.standard_normal(shapes[3]) if eq.endswith("->lmL") else \
        rng.standard_normal((P.shape[0], A.shape[1], Q.shape[0]))
    ops = [dev.from_numpy(o) for o in (P, A, Q, x)]
    ref = np.einsum(eq, P, A, Q, x)
    res = {}
    old_m = lib.ttk_fused_set_mfma(1)
    try:
        for on in (0, 1):
            old = _set_csplit(on)
            try:
                one = dev.read(dev.einsum(eq, *ops, fused=True))
                outs = [dev.from_numpy(np.ones(ref.shape)) for _ in range(2)]
                with dev.einsum_batch():
                    dev.einsum(eq, *ops, out=outs[0], alpha=0.5, beta=2.0, fused=True)
                    dev.einsum(eq, *ops, out=outs[1], fused=True)
                res[on] = (one, dev.read(outs[0]), dev.read(outs[1]))
            finally:
                _set_csplit(old)
    finally:
        lib.ttk_fused_set_mfma(old_m)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(res[1][0] - ref)) <= 1e-13 * scale
    assert np.max(np.abs(res[1][1] - (0.5 * ref + 2.0))) <= 1e-13 * scale


@pytest.mark.gpu
@pytest.mark.parametrize("ineq", [False, True])
def test_schur_mfma_rows_split_bit_identical(dev, ineq):
    """the Schur-reduced operator (two multi-task launches) with wide MFMA rows: split rows (knob on)
    and single-workgroup rows (knob off) give the same matvec bit for bit"""
    from ttipm_amd import tt_ipm
    rng = np.random.default_rng(9)
    r, R, s, S, n = 14, 96, 10, 9, 4
    cls = tt_ipm.IneqMatVecWrapper if ineq else tt_ipm.MatVecWrapper
    L = {k: dev.from_numpy(rng.standard_normal((r, s, r)) * 0.1) for k in cls.keys}
    Am = {k: dev.from_numpy(rng.standard_normal((s, n, n, S)) * 0.1) for k in cls.keys}
    Rr = {k: dev.from_numpy(rng.standard_normal((R, S, R)) * 0.1) for k in cls.keys}
    invI = dev.from_numpy(rng.uniform(0.5, 2.0, (r, n, R)))
    nb = 3 if ineq else 2
    v = dev.from_numpy(rng.standard_normal(nb * r * n * R))
    outs = {}
    for on in (0, 1):
        old = _set_csplit(on)
        try:
            op = cls(L, Am, Rr, invI, (r, n, R))
            assert op.h != 0
            outs[on] = dev.read(op.matvec(v))
        finally:
            _set_csplit(old)
    assert np.array_equal(outs[0], outs[1])


def _set_dual(on):
    import ctypes
    from ttipm_amd import _lib
    old = ctypes.c_int(0)
    assert _lib.lib.ttk_ctx_set_knob(None, _lib.KNOB_APPLY_DUAL, int(on), ctypes.byref(old)) == 0
    return old.value


@pytest.mark.gpu
@pytest.mark.parametrize("ineq", [False, True])
@pytest.mark.parametrize("dims", [(12, 16, 10, 9, 4), (3, 4, 5, 5, 4), (16, 20, 12, 12, 4)])
def test_schur_terms_side_by_side_bit_identical(dev, ineq, dims):
    """the Schur-reduced operator on VALU rows at maxcut sizes: a task's two terms side by side, one
    half of the workgroup each (TTK_KNOB_APPLY_DUAL on, the default), and one after the other (off)
    give the same matvec bit for bit (the sequential form is the one the golden tests pin)"""
    from ttipm_amd import tt_ipm
    rng = np.random.default_rng(11)
    r, R, s, S, n = dims
    cls = tt_ipm.IneqMatVecWrapper if ineq else tt_ipm.MatVecWrapper
    L = {k: dev.from_numpy(rng.standard_normal((r, s, r)) * 0.1) for k in cls.keys}
    Am = {k: dev.from_numpy(rng.standard_normal((s, n, n, S)) * 0.1) for k in cls.keys}
    Rr = {k: dev.from_numpy(rng.standard_normal((R, S, R)) * 0.1) for k in cls.keys}
    invI = dev.from_numpy(rng.uniform(0.5, 2.0, (r, n, R)))
    nb = 3 if ineq else 2
    v = dev.from_numpy(rng.standard_normal(nb * r * n * R))
    outs = {}
    for on in (0, 1):
        old = _set_dual(on)
        try:
            op = cls(L, Am, Rr, invI, (r, n, R))
            assert op.h != 0
            outs[on] = dev.read(op.matvec(v))
        finally:
            _set_dual(old)
    assert np.array_equal(outs[0], outs[1])


def _set_knob(knob, on):
    import ctypes
    from ttipm_amd import _lib
    old = ctypes.c_int(0)
    assert _lib.lib.ttk_ctx_set_knob(None, knob, int(on), ctypes.byref(old)) == 0
    return old.value


@pytest.mark.gpu
@pytest.mark.parametrize("ineq", [False, True])
@pytest.mark.parametrize("dims", [(12, 16, 10, 9, 4), (3, 4, 5, 5, 4), (16, 20, 12, 12, 4), (8, 5, 4, 4, 4),
                                  (14, 96, 10, 9, 4)])
def test_schur_one_launch_bit_identical(dev, ineq, dims):
    """the Schur-reduced operator as ONE launch (TTK_KNOB_SCHUR_ONE, the default: the o1 rows take w
    from the w rows of the same launch over an sc1 hand-off) gives the two-launch matvec bit for bit,
    over many applies in a row (the arrival counter is monotonic across launches), on VALU rows
    (side by side or not) and MFMA rows, and no hand-off wait ever gives up"""
    import ctypes
    from ttipm_amd import _lib, tt_ipm
    rng = np.random.default_rng(13)
    r, R, s, S, n = dims
    cls = tt_ipm.IneqMatVecWrapper if ineq else tt_ipm.MatVecWrapper
    L = {k: dev.from_numpy(rng.standard_normal((r, s, r)) * 0.1) for k in cls.keys}
    Am = {k: dev.from_numpy(rng.standard_normal((s, n, n, S)) * 0.1) for k in cls.keys}
    Rr = {k: dev.from_numpy(rng.standard_normal((R, S, R)) * 0.1) for k in cls.keys}
    invI = dev.from_numpy(rng.uniform(0.5, 2.0, (r, n, R)))
    nb = 3 if ineq else 2
    vs = [dev.from_numpy(rng.standard_normal(nb * r * n * R)) for _ in range(6)]
    to = ctypes.c_uint(0)
    assert _lib.lib.ttk_dep_timeouts(ctypes.byref(to), 1) == 0
    outs = {}
    for on in (0, 1):
        for prep in (0, 1):  # operand images pre-permuted at build (TTK_KNOB_SCHUR_PREP) or gathered
            old, oldp = _set_knob(_lib.KNOB_SCHUR_ONE, on), _set_knob(_lib.KNOB_SCHUR_PREP, prep)
            try:
                op = cls(L, Am, Rr, invI, (r, n, R))
                assert op.h != 0
                res = []
                for v in vs:
                    y = op.matvec(v)
                    res.append(dev.read(op.matvec(y)))  # chained: each apply reads the previous output
                outs[on, prep] = res
            finally:
                _set_knob(_lib.KNOB_SCHUR_ONE, old)
                _set_knob(_lib.KNOB_SCHUR_PREP, oldp)
    for key in outs:
        for a, b in zip(outs[0, 0], outs[key]):
            assert np.array_equal(a, b), key
    assert _lib.lib.ttk_dep_timeouts(ctypes.byref(to), 0) == 0 and to.value == 0


@pytest.mark.gpu
@pytest.mark.parametrize("ineq", [False, True])
@pytest.mark.parametrize("mw_min", [0, 16384])
def test_lgmres_one_launch_arnoldi_bit_identical(dev, ineq, mw_min):
    """whole LGMRES solves on a Schur operator: the multi-workgroup Arnoldi step as ONE launch
    (TTK_KNOB_ARNOLDI_ONE) and as three launches (the default since round 6) give the same solution, residual and
    iteration count bit for bit (mw_min 0: every step on the multi-workgroup path; 16384: the
    default split), with the one-launch Schur matvec on and off, and no hand-off wait gives up"""
    import ctypes
    from ttipm_amd import _lib, lgmres, tt_ipm
    rng = np.random.default_rng(17)
    r, R, s, S, n = 9, 12, 4, 4, 4
    cls = tt_ipm.IneqMatVecWrapper if ineq else tt_ipm.MatVecWrapper
    L = {k: dev.from_numpy(rng.standard_normal((r, s, r)) * 0.3) for k in cls.keys}
    Am = {k: dev.from_numpy(rng.standard_normal((s, n, n, S)) * 0.3) for k in cls.keys}
    Rr = {k: dev.from_numpy(rng.standard_normal((R, S, R)) * 0.3) for k in cls.keys}
    invI = dev.from_numpy(rng.uniform(0.5, 2.0, (r, n, R)))
    nb = 3 if ineq else 2
    b = dev.from_numpy(rng.standard_normal(nb * r * n * R))
    m = r * n * R
    to = ctypes.c_uint(0)
    assert _lib.lib.ttk_dep_timeouts(ctypes.byref(to), 1) == 0
    res = {}
    old_mw = _set_knob(_lib.KNOB_LGMRES_MW_MIN, mw_min)
    try:
        for arn in (0, 1):
            for one in (0, 1):
                o1, o2 = _set_knob(_lib.KNOB_ARNOLDI_ONE, arn), _set_knob(_lib.KNOB_SCHUR_ONE, one)
                try:
                    op = cls(L, Am, Rr, invI, (r, n, R))
                    info = {}
                    x = lgmres.lgmres(op.matvec_into, b, rtol=1e-10, max_it=300, restart=min(m, 100),
                                      augment=max(min(m, 100) // 10, 3), info=info, native=op.h)
                    res[arn, one] = (dev.read(x), info["its"], info["res"], info["reason"])
                finally:
                    _set_knob(_lib.KNOB_ARNOLDI_ONE, o1)
                    _set_knob(_lib.KNOB_SCHUR_ONE, o2)
    finally:
        _set_knob(_lib.KNOB_LGMRES_MW_MIN, old_mw)
    ref = res[0, 0]
    assert ref[1] > 10
    for k, v in res.items():
        assert np.array_equal(v[0], ref[0]) and v[1:] == ref[1:], k
    assert _lib.lib.ttk_dep_timeouts(ctypes.byref(to), 0) == 0 and to.value == 0


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(212, 64, 2544), (60, 44, 2700), (116, 64, 1160), (33, 7, 300), (240, 60, 1000)])
def test_splitk_one_launch_bit_identical(dev, shape):
    """The one-launch split-K GEMM (TTK_KNOB_SPLITK_FUSED: partial tiles handed to the last-arriving
    split block over write-through stores and an arrival counter) equals the split kernel + reduce
    kernel bit for bit, with alpha / beta, on batched operands, and leaves its counters reset (the
    same call repeated gives the same bits)."""
    import torch
    from ttipm_amd import _lib
    from ttipm_amd import dev as D
    M, N, K = shape
    g = torch.Generator("cuda").manual_seed(M * N + K)
    a = torch.randn(2, M, K, dtype=torch.float64, device="cuda", generator=g)
    b = torch.randn(2, K, N, dtype=torch.float64, device="cuda", generator=g)
    c0 = torch.randn(2, M, N, dtype=torch.float64, device="cuda", generator=g)
    outs = []
    for fused in (0, 1, 1):
        old = _set_knob(_lib.KNOB_SPLITK_FUSED, fused)
        try:
            c = D.clone(c0)
            D.einsum("bmk,bkn->bmn", a, b, out=c, alpha=0.75, beta=-1.25)
            outs.append(D.read(c))
        finally:
            _set_knob(_lib.KNOB_SPLITK_FUSED, old)
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])
    ref = 0.75 * np.einsum("bmk,bkn->bmn", D.read(a), D.read(b)) - 1.25 * D.read(c0)
    assert np.allclose(outs[0], ref, rtol=1e-11, atol=1e-10)
