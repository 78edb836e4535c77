"""Golden-vector generation shim for petsc4py 3.25.1 (absent from the image).

Implements exactly the surface `src/tt_ipm.py:101-162` touches: `PETSc.KSP().create`,
`setType('lgmres')`, `PETSc.Options().setValue`, `setFromOptions`, a MATPYTHON shell
(`Mat().createPython` + `setPythonContext` whose `mult(self, mat, x, y)` writes `y.array_w`),
`Vec().createWithArray`, `ksp.solve(b, x)`.  The solve itself is `oracle/petsc_lgmres.py`,
a restatement of PETSc's KSPLGMRES.  Used ONLY by tests/golden/make_golden.py."""
import os
import sys

import numpy as np

_here = os.path.dirname(os.path.abspath(__file__))
_repo = os.path.abspath(os.path.join(_here, "..", "..", "..", ".."))
if _repo not in sys.path:
    sys.path.insert(0, _repo)
from oracle.petsc_lgmres import lgmres  # noqa: E402


def init(*a, **k):
    return None


class _PETSc:
    COMM_WORLD = object()
    _opts = {}

    class Options:
        def setValue(self, k, v):
            _PETSc._opts[k.lstrip('-')] = v

    class Vec:
        def createWithArray(self, arr, comm=None):
            self.arr = arr
            return self

        @property
        def array_r(self):
            return self.arr

        @property
        def array_w(self):
            return self.arr

        def destroy(self):
            pass

    class Mat:
        def createPython(self, shape, comm=None):
            self.shape = shape
            return self

        def setPythonContext(self, ctx):
            self.ctx = ctx

        def setUp(self):
            pass

    class KSP:
        def create(self, comm=None):
            return self

        def setType(self, t):
            assert t == "lgmres"

        def setFromOptions(self):
            o = _PETSc._opts
            self.restart = int(o.get("ksp_gmres_restart", 30))
            self.augment = int(o.get("ksp_lgmres_augment", 2))
            self.rtol = float(o.get("ksp_rtol", 1e-5))
            self.max_it = int(o.get("ksp_max_it", 10000))

        def setOperators(self, A):
            self.A = A

        def solve(self, b, x):
            ctx = self.A.ctx
            n = b.arr.size

            def mv(v):
                xin = _PETSc.Vec().createWithArray(np.array(v, copy=True))
                yout = _PETSc.Vec().createWithArray(np.empty(n))
                ctx.mult(None, xin, yout)
                return np.array(yout.arr, copy=True)

            x.arr[:] = lgmres(mv, b.arr, rtol=self.rtol, max_it=self.max_it, restart=self.restart,
                              augment=self.augment)

        def destroy(self):
            pass


PETSc = _PETSc
sys.modules.setdefault("petsc4py.PETSc", _PETSc)
