import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D
from ttipm_amd._lib import lib

cases = [
    ("lsr,smnS,LSR,rnR->lmL", ((1, 1, 1), (1, 4, 4, 3), (5, 3, 5), (1, 4, 5)), ((1, 1, 1), (48, 12, 3, 1), (15, 5, 1), (60, 5, 1)), ((1, 4, 5), (60, 5, 1))),
    ("lsr,smnS,LSR,rnR->lmL", ((9, 2, 9), (2, 4, 4, 2), (6, 2, 6), (9, 4, 6)), ((18, 9, 1), (32, 8, 2, 1), (12, 6, 1), (72, 6, 1)), ((9, 4, 6), (72, 6, 1))),
    ("lsr,smnS,LSR,lmL->rnR", ((8, 1, 8), (1, 4, 4, 1), (3, 1, 3), (8, 4, 3)), ((8, 8, 1), (16, 4, 1, 1), (3, 3, 1), (36, 3, 1)), ((8, 4, 3), (36, 3, 1))),
]
rng = np.random.default_rng(0)
for eq, shapes, strides, (osh, ost) in cases:
    ops = []
    for sh, st in zip(shapes, strides):
        n = 1 + sum((e - 1) * s for e, s in zip(sh, st))
        base = D.from_numpy(rng.standard_normal(n + 64))
        ops.append(torch.as_strided(base, sh, st))
    n = 1 + sum((e - 1) * s for e, s in zip(osh, ost))
    obase = D.from_numpy(rng.standard_normal(n + 64))
    out = torch.as_strided(obase, osh, ost)
    o0 = D.read(out).copy()
    ref = np.einsum(eq, *[D.read(o) for o in ops]) + o0
    D.einsum(eq, *ops, out=out, beta=1.0)
    f = D.read(out)
    out2 = torch.as_strided(D.from_numpy(D.read(obase) * 0), osh, ost)
    D.copy_(out2, D.from_numpy(o0))
    old = lib.ttk_einsum_set_fused(0)
    D.einsum(eq, *ops, out=out2, beta=1.0)
    lib.ttk_einsum_set_fused(old)
    p = D.read(out2)
    print(eq, shapes[1], "fused err", np.abs(f - ref).max() / np.abs(ref).max(), "plain err", np.abs(p - ref).max() / np.abs(ref).max())
