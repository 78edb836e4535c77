"""Loader for the reference's local KKT solve fixtures (`tests/golden/local.npz`, written by
`tests/golden/make_local.py` from `_ipm_local_solver(_ineq)`, src/tt_ipm.py:183-401).

`load(name, wrap, block_matrix, view)` rebuilds one recorded call's arguments: `wrap` turns a
NumPy array into the caller's tensor type (identity for the oracle, device upload for the HIP
path), `block_matrix()` makes an empty block matrix and `view(bm)` its core-0 view."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "local.npz"))
CASES = [str(c) for c in G["cases"]]


def _pair(s):
    return int(s[0]), int(s[1])


def load(name, wrap, block_matrix, view, set_block, add_alias):
    keys = [tuple(int(v) for v in k) for k in G[f"{name}/keys"]]
    XL, XR, bL, bR, b = {}, {}, {}, {}, {}
    for f in G.files:
        if not f.startswith(name + "/"):
            continue
        tail = f[len(name) + 1:]
        if tail.startswith("XL"):
            XL[_pair(tail[2:])] = wrap(G[f])
        elif tail.startswith("XR"):
            XR[_pair(tail[2:])] = wrap(G[f])
        elif tail.startswith("bL"):
            bL[int(tail[2:])] = wrap(G[f])
        elif tail.startswith("bR"):
            bR[int(tail[2:])] = wrap(G[f])
        elif tail[0] == "b" and tail[1:].isdigit():
            b[int(tail[1:])] = wrap(G[f])
    bm = block_matrix()
    for k in keys:  # the reference's block order (it sets the accumulation order)
        set_block(bm, k, wrap(G[f"{name}/A{k[0]}{k[1]}"]))
    for row in G[f"{name}/transposes"]:
        add_alias(bm, (int(row[0]), int(row[1])), (int(row[2]), int(row[3])), True)
    for row in G[f"{name}/aliases"]:
        add_alias(bm, (int(row[0]), int(row[1])), (int(row[2]), int(row[3])), False)
    XL = {k: XL[k] for k in keys if k in XL} | {k: v for k, v in XL.items() if k not in keys}
    XR = {k: XR[k] for k in keys if k in XR} | {k: v for k, v in XR.items() if k not in keys}
    args = (XL, view(bm), XR, bL, dict(sorted(b.items())), bR, wrap(G[f"{name}/prev"]),
            int(G[f"{name}/size_limit"]), bool(G[f"{name}/dense_solve"]))
    expect = {k: G[f"{name}/{k}"] for k in ("sol", "rhs")}
    expect.update({k: float(G[f"{name}/{k}"]) for k in ("res_old", "res_min", "nrhs")})
    expect["failed"] = bool(G[f"{name}/failed"])
    expect["exc"] = str(G[f"{name}/exc"])
    return args, expect


def is_ineq(name):
    return name.startswith("ineq")


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(np.max(np.abs(b)), 1e-300))
