"""Diagnostics (GPU): run a solve with every fused local apply / environment batch / Schur operator
application recomputed with the MFMA stages switched off (pairwise plan), and report the first
call whose results differ by more than 1e-10 relative or are not finite.

    python tools/check_mfma.py graphm graphm_3 256 2 [assemblies]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402

from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd import tt_als, tt_ipm  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg_name, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
nmax = int(sys.argv[5]) if len(sys.argv) > 5 else 3
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(HERE), "configs", cfg_name + ".yaml")))
stats = {"calls": 0, "bad": 0}


def _cmp(tag, a, b, info):
    stats["calls"] += 1
    a, b = D.read(a), D.read(b)
    scale = max(np.max(np.abs(b)), 1e-300) if b.size else 1.0
    err = np.max(np.abs(a - b)) / scale if b.size else 0.0
    if not np.all(np.isfinite(a)) or err > 1e-10:
        stats["bad"] += 1
        if stats["bad"] <= 5:
            print(f"MISMATCH {tag}: rel err {err:.3e} finite={np.all(np.isfinite(a))} {info}", flush=True)


orig_env = tt_als.env_update_many


def env_checked(backward, items):
    got = orig_env(backward, items)
    old = lib.ttk_fused_set_mfma(0)
    try:
        ref = orig_env(backward, items)
    finally:
        lib.ttk_fused_set_mfma(old)
    for i, (g, r) in enumerate(zip(got, ref)):
        P, x, A, y = items[i]
        _cmp("env", g, r, (backward, tuple(P.shape), tuple(x.shape), tuple(A.shape), tuple(A.stride()), tuple(y.shape)))
    return got


tt_als.env_update_many = env_checked
orig_einsum = D.einsum


def einsum_checked(eq, *ops, out=None, alpha=1.0, beta=0.0, fused=False, algo=None):
    if not fused or D._TL.batch[0]:
        return orig_einsum(eq, *ops, out=out, alpha=alpha, beta=beta, fused=fused, algo=algo)
    keep = None if out is None else D.clone(out)
    got = orig_einsum(eq, *ops, out=out, alpha=alpha, beta=beta, fused=fused, algo=algo)
    old = lib.ttk_fused_set_mfma(0)
    try:
        ref = orig_einsum(eq, *ops, out=None if keep is None else keep, alpha=alpha, beta=beta, fused=fused)
    finally:
        lib.ttk_fused_set_mfma(old)
    _cmp("einsum " + eq, got, ref, [tuple(o.shape) for o in ops] + [tuple(o.stride()) for o in ops])
    return got


D.einsum = einsum_checked
for _m in (tt_ipm, tt_als):
    if hasattr(_m, "einsum"):
        _m.einsum = einsum_checked
if os.environ.get("NOBATCH"):
    class _NoBatch:
        def __enter__(self):
            return self

        def __exit__(self, *exc):
            return False

    D.einsum_batch = _NoBatch


def _wrap_mv(cls):
    orig = cls.matvec_into

    def mv(self, v, out):
        got = orig(self, v, out)
        if not self.h:
            return got
        ref = D.empty(v.numel())
        h, self.h = self.h, 0
        old = lib.ttk_fused_set_mfma(0)
        try:
            orig(self, v, ref)
        finally:
            lib.ttk_fused_set_mfma(old)
            self.h = h
        _cmp("schur " + cls.__name__, got, ref, [tuple(t.shape) for t in self.L.values()] if isinstance(self.L, dict) else "")
        return got
    cls.matvec_into = mv


_wrap_mv(tt_ipm.MatVecWrapper)
_wrap_mv(tt_ipm.IneqMatVecWrapper)


class _Stop(Exception):
    pass


class Trace(list):
    def append(self, item):
        super().append(item)
        print("assembly", len(self), {k: item[k] for k in ("mu", "primal_error", "dual_error")}, flush=True)
        if len(self) >= nmax:
            raise _Stop


torch.cuda.set_device(0)
try:
    run_and_record(prob, cfg, seed, rank, trace=Trace(), verbose=False)
except _Stop:
    pass
except (ZeroDivisionError, FloatingPointError, ArithmeticError) as e:
    print("solve stopped:", repr(e))
print("checked", stats)
