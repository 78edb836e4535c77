"""Golden-vector generation shim for opt_einsum 3.4.0 (absent from the image).

opt_einsum only chooses the pairwise contraction order; the sums are the same.  This shim
executes `contract` / `contract_expression` with numpy.einsum's greedy planner (cached per
equation+shapes), or the explicit path when one is given.  Used ONLY by make_golden.py."""
from functools import lru_cache

import numpy as np


@lru_cache(maxsize=4096)
def _greedy(eq, shapes):
    return np.einsum_path(eq, *[np.empty(s) for s in shapes], optimize="greedy")[0]


def contract(eq, *ops, optimize="greedy", **kw):
    if isinstance(optimize, (list, tuple)):
        path = ["einsum_path"] + [tuple(p) for p in optimize]
    else:
        path = _greedy(eq, tuple(o.shape for o in ops))
    return np.einsum(eq, *ops, optimize=path)


def contract_expression(eq, *shapes, optimize="greedy", **kw):
    path = _greedy(eq, tuple(tuple(s) for s in shapes))
    return lambda *ops: np.einsum(eq, *ops, optimize=path)
