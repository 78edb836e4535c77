"""Import alias: exposes the package directory `tensor-train-interior-point-method_amd/` (whose
name is not a Python identifier) as the importable package `ttipm_amd`."""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "tensor-train-interior-point-method_amd")]
_init = _os.path.join(__path__[0], "__init__.py")
with open(_init) as _f:
    exec(compile(_f.read(), _init, "exec"))
