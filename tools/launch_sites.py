"""Diagnostics (GPU): which Python call sites issue the library's kernel launches during one solve.
Every ttk_* entry point is wrapped to record its Python call site (innermost package frames) and the
launches it issued (ttk_launch_count delta); prints the sites by launches per IPM iteration.

    python tools/launch_sites.py maxcut maxcut_10 41 1 [frames]"""
import collections
import os
import sys
import traceback
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd import _lib  # noqa: E402
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg_name, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
depth = int(sys.argv[5]) if len(sys.argv) > 5 else 3
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                                       cfg_name + ".yaml")))
calls = collections.Counter()
launches = collections.Counter()
by_fn = collections.Counter()
count = _lib.lib.ttk_launch_count


DEPTH = [0]


class _Wrap:
    """outermost wrapped call only (dev.* functions call each other and the library)"""
    def __init__(self, name, f):
        self.name, self.f = name, f

    def __call__(self, *a, **k):
        if DEPTH[0]:
            return self.f(*a, **k)
        DEPTH[0] += 1
        n0 = count()
        try:
            r = self.f(*a, **k)
        finally:
            DEPTH[0] -= 1
        d = count() - n0
        if d:
            fr = [f for f in traceback.extract_stack()[:-1]
                  if ("ttipm" in f.filename or "interior-point" in f.filename) and not f.filename.endswith("dev.py")]
            site = " < ".join(reversed([f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-depth:]]))
            calls[(self.name, site)] += 1
            launches[(self.name, site)] += d
            by_fn[self.name] += d
        return r


# the _ttkbind packer holds raw pointers to these three: leave them, their launches are attributed to
# the dev.* function that issued them
BOUND = ("ttk_einsum", "ttk_copy_nd", "ttk_mul_nd", "ttk_axpby_nd", "ttk_normalize", "ttk_scale_axis_ss", "ttk_dot_nd_dev",
         "ttk_fill", "ttk_env_update")
for n in [n for n in dir(_lib.lib) if n.startswith("ttk_") and n != "ttk_launch_count" and n not in BOUND]:
    try:
        setattr(_lib.lib, n, _Wrap(n, getattr(_lib.lib, n)))
    except AttributeError:
        pass
for n, f in list(vars(D).items()):
    if isinstance(f, types.FunctionType) and f.__module__ == D.__name__ and not n.startswith("__"):
        setattr(D, n, _Wrap("dev." + n, f))
run_and_record(prob, cfg, seed, rank, verbose=False)  # warm
calls.clear(), launches.clear(), by_fn.clear()
l0 = count()
r = run_and_record(prob, cfg, seed, rank, verbose=False)
tot = count() - l0
it = r["num_iters"]
print(f"iters {it}  launches {tot} ({tot / it:.0f} per IPM iteration; {sum(by_fn.values()) / it:.0f} through wrapped "
      "entry points, the rest from the _ttkbind packer)")
print("by entry point:")
for n, c in by_fn.most_common(25):
    print(f"{c / it:9.1f}/it  {n}")
print("by call site:")
for k, c in launches.most_common(60):
    print(f"{c / it:9.1f}/it  ({calls[k] / it:7.1f} calls/it)  {k[0]:26s} {k[1]}")
