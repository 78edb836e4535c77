"""The native step-size eigen-ALS orchestration (`_ttkbind.eig_als`, csrc/ttk_host_eig.inc) on CPU: its
host logic -- sweep control, deferred residuals, truncation rule, kicks from the restated MT19937
Gaussian stream, the bail-out to Python -- against tt_eig.py's Python orchestration of the same
`tt_max_generalised_eigen` (`src/tt_als.py:1132-1283`), with the libttk C ABI replaced by the NumPy
emulator (tests/emu_ttk.py) for BOTH: the binder calls the emulator through C function pointers
(ctypes callbacks), the Python path calls it directly.  Same inputs, same random state: the step,
the solution cores and the random state afterwards must agree bit for bit.  Inputs are the
reference's recorded calls (tests/golden/step.npz).  The device run of the same comparison is
tests/test_gpu_step.py::test_native_eigen_als_bit_identical_to_python."""
import ctypes
import glob
import importlib.util
import os

import numpy as np
import pytest

from tests import step_cases as SC
from tests.emu_ttk import emulated_ttipm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DESC_WORDS = 8 * 34 + 20  # the binder's einsum descriptor (csrc/ttk_host_bind.cpp)


@pytest.fixture(scope="module")
def pkg():
    return emulated_ttipm()


@pytest.fixture(scope="module")
def native(pkg):
    """_ttkbind bound to the emulator: every libttk entry point the binder and eig_als call becomes a
    ctypes callback into tests/emu_ttk.py with the C signature of ttipm_amd._lib._SIGS."""
    paths = glob.glob(os.path.join(ROOT, "tensor-train-interior-point-method_amd", "_ttkbind*.so"))
    if not paths:
        pytest.skip("_ttkbind not built (run __graft_entry__.build())")
    spec = importlib.util.spec_from_file_location("_ttkbind", paths[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from ttipm_amd import _lib as L
    lib = L.lib
    keep = []

    def cb(name, fn=None):
        res, args = L._SIGS[name]
        # looked up at call time, so a test that patches the emulator patches both paths
        c = ctypes.CFUNCTYPE(res, *args)(fn or (lambda *a: getattr(lib, name)(*a)))
        keep.append(c)
        return ctypes.cast(c, ctypes.c_void_p).value

    def einsum(s, eq, desc, out, alpha, beta):
        return lib.ttk_einsum(s, eq, (ctypes.c_int64 * DESC_WORDS).from_address(desc), out, alpha, beta)

    def ray_sync(s, v, Mv, n, ev_out, r2_out):
        e, r = ctypes.c_double(0.0), ctypes.c_double(0.0)
        rc = lib.ttk_rayleigh_tail_sync(s, v, Mv, n, ctypes.byref(e), ctypes.byref(r))
        ev_out[0], r2_out[0] = e.value, r.value
        return rc

    b1 = (cb("ttk_einsum", einsum), cb("ttk_copy_nd"), cb("ttk_mul_nd"), 0)
    b2 = (cb("ttk_axpby_nd"), cb("ttk_normalize"), cb("ttk_scale_axis_ss"), cb("ttk_dot_nd_dev"), cb("ttk_fill"))
    b3 = [cb(n) if n != "ttk_rayleigh_tail_sync" else cb(n, ray_sync) for n in (
        "ttk_svd_work", "ttk_svd_tol", "ttk_qr_work", "ttk_qr", "ttk_syev_extreme_work", "ttk_syev_extreme",
        "ttk_read_sync", "ttk_upload", "ttk_cholesky_sync", "ttk_trsm_lower", "ttk_rayleigh_tail_dev",
        "ttk_rayleigh_tail_sync", "ttk_einsum_batch_begin", "ttk_einsum_batch_end", "ttk_svd_tol_read")]

    def rebind():  # the binder's entry points are process-wide: (re)bind before each use
        mod.bind(*b1)
        mod.bind2(*b2)
        mod.bind_eig(b3)
        return mod

    rebind._keep = keep  # the callbacks live as long as the fixture
    return rebind


def _run(E, D, case, use, size_limit=256):
    A, Dl, x0, st, _, _ = SC.call(case)
    np.random.set_state(st)
    up = (lambda tt: None if tt is None else [D.from_numpy(c) for c in tt])
    old = E._native_eig
    E._native_eig = lambda: use
    try:
        s, x = E.tt_max_generalised_eigen(up(A), up(Dl), x0=up(x0), tol=1e-8, size_limit=size_limit)
    finally:
        E._native_eig = old
    return s, [D.to_numpy(c).copy() for c in x], np.random.get_state()


def _same(a, b):
    (s0, x0, r0), (s1, x1, r1) = a, b
    assert s0 == s1, (s0, s1)
    assert [c.shape for c in x0] == [c.shape for c in x1]
    assert all(np.array_equal(u, v) for u, v in zip(x0, x1))
    assert np.array_equal(r0[1], r1[1]) and r0[2:] == r1[2:]


@pytest.mark.parametrize("case", ["s41_c0", "s41_c1", "s14_c16", "s14_c17"])
def test_native_eigen_als_matches_python_on_emulator(pkg, native, case):
    from ttipm_amd import dev as D
    from ttipm_amd import tt_eig as E
    n0 = E.NATIVE_CALLS["native"]
    py = _run(E, D, case, None)
    nat = _run(E, D, case, native())
    assert E.NATIVE_CALLS["native"] == n0 + 1  # the native path ran (no bail-out)
    _same(py, nat)
    ref = SC.call(case)[4]
    assert abs(nat[0] - ref) <= 1e-10 * ref, (nat[0], ref)  # and it is the reference's step


def test_native_eigen_als_bails_out_to_python(pkg, native):
    """size_limit 1 sends every two-site solve to the LOBPCG branch, which only the Python path has:
    the native call returns status 1 with nothing changed and the call reruns in Python from the same
    random state -- the result is the Python path's, bit for bit."""
    from ttipm_amd import dev as D
    from ttipm_amd import tt_eig as E
    b0, n0 = E.NATIVE_CALLS["bail"], E.NATIVE_CALLS["native"]
    py = _run(E, D, "s41_c0", None, size_limit=1)
    nat = _run(E, D, "s41_c0", native(), size_limit=1)
    assert E.NATIVE_CALLS["bail"] == b0 + 1 and E.NATIVE_CALLS["native"] == n0
    _same(py, nat)


def test_native_eigen_als_generalised_branch_failure(pkg, native):
    """The generalised-eigenproblem branch's failure path (`_gen_max_eig` raising: A not positive
    definite -> keep the previous vector, step *= 1 - eps; `src/tt_als.py:986-996`): with the emulated
    Cholesky failing every time, every negative-eigenvalue local solve of s41_c0 takes it (109 of them
    once the first failures have changed the path), in both orchestrations, bit for bit."""
    from ttipm_amd import _lib as L
    from ttipm_amd import dev as D
    from ttipm_amd import tt_eig as E
    lib = L.lib
    real = type(lib).ttk_cholesky_sync

    def fail(self, s, A, n):
        self.err = b"not positive definite (forced)"
        return 3

    type(lib).ttk_cholesky_sync = fail
    try:
        calls = []
        og = E._gen_max_eig

        def counted(*a):
            calls.append(1)
            return og(*a)

        E._gen_max_eig = counted
        try:
            py = _run(E, D, "s41_c0", None)
        finally:
            E._gen_max_eig = og
        assert len(calls) >= 9  # every negative-eigenvalue solve fails over (the path then changes)
        nat = _run(E, D, "s41_c0", native())
    finally:
        type(lib).ttk_cholesky_sync = real
    _same(py, nat)


def test_native_eigen_als_zero_step_raises_like_python(pkg, native):
    """A generalised eigenvalue of the wrong sign makes the step max(0, 1/lam) = 0, and the residual's
    A / step then raises ZeroDivisionError in the Python orchestration (as in the reference).  The native
    call bails out on it (status 1, nothing changed) and the Python rerun raises the same exception."""
    from ttipm_amd import _lib as L
    from ttipm_amd import dev as D
    from ttipm_amd import tt_eig as E
    lib = L.lib
    real = type(lib).ttk_syev_extreme

    def flipped(self, s, A, n, which, ev, vec, work):
        rc = real(self, s, A, n, which, ev, vec, work)
        if which:  # the largest eigenpair: only _gen_max_eig asks for it
            from tests.emu_ttk import _dv
            _dv(ev, 1)[0] = -abs(_dv(ev, 1)[0]) - 1.0
        return rc

    type(lib).ttk_syev_extreme = flipped
    try:
        with pytest.raises(ZeroDivisionError):
            _run(E, D, "s41_c0", None)
        b0 = E.NATIVE_CALLS["bail"]
        with pytest.raises(ZeroDivisionError):
            _run(E, D, "s41_c0", native())
        assert E.NATIVE_CALLS["bail"] == b0 + 1
    finally:
        type(lib).ttk_syev_extreme = real
