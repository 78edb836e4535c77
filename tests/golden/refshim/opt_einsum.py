"""Golden-vector generation shim for opt_einsum 3.4.0 (absent from the image).

`contract_expression(eq, *shapes, optimize='greedy')` and `contract` evaluate through
`oracle/opt_einsum_greedy.py`, a restatement of opt_einsum 3.4.0's greedy path (memory_limit=None)
and its tensordot/einsum execution, so the reference runs with the pairwise contraction order it
has in its own environment.  Used ONLY by make_golden.py."""
import os
import sys

import numpy as np

_repo = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
if _repo not in sys.path:
    sys.path.insert(0, _repo)
from oracle.opt_einsum_greedy import contract as _contract  # noqa: E402


def contract(eq, *ops, optimize="greedy", **kw):
    if isinstance(optimize, (list, tuple)):  # explicit path: plain pairwise numpy execution
        return np.einsum(eq, *ops, optimize=["einsum_path"] + [tuple(p) for p in optimize])
    return _contract(eq, *ops)


def contract_expression(eq, *shapes, optimize="greedy", **kw):
    return lambda *ops: _contract(eq, *ops)
