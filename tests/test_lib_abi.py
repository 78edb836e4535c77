"""The C ABI: every function `include/ttk.h` declares is exported by the built libttk.so and bound
by the host layer (`ttipm_amd._lib`).  CPU-only (loads the library, calls nothing on a device)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tensor-train-interior-point-method_amd", "libttk.so")


def _declared():
    txt = open(os.path.join(ROOT, "include", "ttk.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ttk_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_api():
    names = _declared()
    for must in ("ttk_gemm_offs", "ttk_svd", "ttk_qr", "ttk_lu_sync", "ttk_cholesky_sync", "ttk_syev_extreme",
                 "ttk_lgmres_arnoldi_sync", "ttk_contract_stats"):
        assert must in names


@pytest.mark.skipif(not os.path.exists(SO), reason="libttk.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(SO)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_host_layer_binds_every_declared_symbol():
    src = open(os.path.join(ROOT, "tensor-train-interior-point-method_amd", "_lib.py")).read()
    unbound = [n for n in _declared() if f'"{n}"' not in src]
    assert not unbound, unbound


def test_product_has_no_cpu_fallback():
    """The product package never imports the oracle and fails loudly without the HIP library."""
    pkg = os.path.join(ROOT, "tensor-train-interior-point-method_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            s = open(os.path.join(pkg, f)).read()
            assert "import oracle" not in s and "from oracle" not in s, f
    lib_src = open(os.path.join(pkg, "_lib.py")).read()
    assert "raise" in lib_src and "libttk" in lib_src


def _bind_module():
    import glob
    import importlib.util
    paths = glob.glob(os.path.join(ROOT, "tensor-train-interior-point-method_amd", "_ttkbind*.so"))
    if not paths:
        pytest.skip("_ttkbind not built (run __graft_entry__.build())")
    spec = importlib.util.spec_from_file_location("_ttkbind", paths[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_native_packer_matches_python_descriptor():
    """csrc/ttk_host_bind.cpp builds the same `ttk_einsum` / `ttk_copy_nd` argument records as the
    Python packer in dev.py; checked by binding recording callbacks instead of libttk (no device)."""
    import torch
    mod = _bind_module()
    seen = {}
    EIN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64),
                           ctypes.c_void_p, ctypes.c_double, ctypes.c_double)
    CPY = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                           ctypes.POINTER(ctypes.c_int64), ctypes.c_double, ctypes.c_double)

    def ein(stream, eq, desc, out, alpha, beta):
        n = desc[0] & 255
        pos, recs = 1, []
        for _ in range(n):
            nd = desc[pos + 1]
            recs.append([desc[pos + k] for k in range(2 + 2 * nd)])
            pos += 2 + 2 * nd
        has_out = desc[pos]
        tail = [desc[pos + k] for k in range(2 + desc[pos + 1])] if has_out else [0]
        seen["ein"] = (eq.decode(), desc[0], recs, tail, out, alpha, beta)
        return 0

    def cpy(stream, src, dst, nd, shp, ss, ds, alpha, beta):
        seen["cpy"] = (src, dst, [shp[i] for i in range(nd)], [ss[i] for i in range(nd)],
                       [ds[i] for i in range(nd)], alpha, beta)
        return 0

    fe, fc = EIN(ein), CPY(cpy)
    addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    mod.bind(addr(fe), addr(fc), addr(fc), 0)
    a = torch.zeros(3, 4, 5, dtype=torch.float64)
    b = torch.zeros(5, 4, 2, dtype=torch.float64).permute(2, 1, 0)
    res = mod.einsum("abc,dbc->ad", [a, b], None, 2.0, 0.5, 256)
    eq, d0, recs, tail, out, alpha, beta = seen["ein"]
    assert eq == "abc,dbc->ad" and d0 == 2 | 256 and tail == [0]
    assert recs[0] == [a.data_ptr(), 3, 3, 4, 5, 20, 5, 1]
    assert recs[1] == [b.data_ptr(), 3, 2, 4, 5] + list(b.stride())
    assert tuple(res.shape) == (3, 2) and out == res.data_ptr() and alpha == 2.0 and beta == 0.0
    o = torch.zeros(2, 3, dtype=torch.float64).t()
    mod.einsum("abc,dbc->ad", [a, b], o, 1.0, 1.0, 0)
    assert seen["ein"][3] == [1, 2] + list(o.stride()) and seen["ein"][6] == 1.0
    src = torch.zeros(4, 6, dtype=torch.float64)[:, 1:5]
    dst = torch.zeros(4, 4, dtype=torch.float64)
    mod.copy_(dst, src, -1.0, 1.0)
    assert seen["cpy"] == (src.data_ptr(), dst.data_ptr(), [4, 4], [6, 1], [4, 1], -1.0, 1.0)


def test_native_gaussian_stream_matches_numpy():
    """csrc/ttk_host_eig.inc restates RandomState.randn (MT19937, polar Gaussian with its cached
    second value) for the eigen-ALS kicks: the same draws and the same state afterwards as NumPy's,
    from states with and without a cached value and across the 624-word regeneration."""
    import numpy as np
    mod = _bind_module()
    for seed in range(24):
        R = np.random.RandomState(seed)
        R.randn(seed * 7 + 1)
        st = R.get_state()
        n = (1, 3, 700, 5000)[seed % 4]
        out, key, pos, hg, g = mod.legacy_randn(st[1], st[2], st[3], st[4], n)
        ref = R.randn(n)
        st2 = R.get_state()
        assert np.array_equal(out, ref), seed
        assert np.array_equal(key, st2[1]) and (pos, hg, g) == (st2[2], st2[3], st2[4]), seed


def test_native_prune_matches_host_rule():
    """The native truncation rule equals tt_ops.prune_singular_vals (cy_src/tt_ops_cy.pyx:161-177) on
    random spectra, exact zeros, empty input and tails straddling eps^2."""
    import numpy as np

    def rule(s, eps):  # tt_ops.prune_singular_vals, restated here to keep this test device-free
        if np.linalg.norm(s) == 0.0:
            return 1
        sc = np.cumsum(np.abs(s[::-1]) ** 2)[::-1]
        r = max(int(np.argmax(sc < eps ** 2)), 1)
        return s.size if sc[-1] > eps ** 2 else r

    mod = _bind_module()
    rs = np.random.RandomState(3)
    cases = [(np.zeros(4), 1e-9), (np.zeros(0), 1e-9), (np.array([1.0, 1e-5, 1e-9]), 1e-9),
             (np.array([1.0, 1e-9]), 1e-9)]
    for _ in range(3000):
        n = rs.randint(1, 40)
        s = np.sort(np.abs(rs.randn(n)) * 10.0 ** rs.uniform(-12, 1, n))[::-1].copy()
        cases.append((s, 10.0 ** rs.uniform(-10, -2) / np.sqrt(rs.randint(2, 14))))
    for s, eps in cases:
        assert mod.prune_singular_vals(s, eps) == rule(s, eps), (s, eps)
