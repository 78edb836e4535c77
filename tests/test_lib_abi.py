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
