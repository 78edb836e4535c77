"""Time `ttk_round` (tt_ops.tt_rank_reduce / _tail_rank_reduce on the native path) on trains shaped
like the IPM's: d cores of (r, 2, 2, r).  Prints per-call latency and a digest of the rounded cores,
so two libraries (TTK_LIB_PATH) can be compared for speed and for identical bits.

    python tools/bench_round.py [reps]
"""
import hashlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd import tt_ops as T  # noqa: E402


def train(rng, ranks):
    return [D.from_numpy(rng.standard_normal((ranks[k], 2, 2, ranks[k + 1])) * (0.5 ** np.arange(ranks[k + 1])))
            for k in range(len(ranks) - 1)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rng = np.random.default_rng(5)
    cases = {"d10_r8": [1] + [8] * 9 + [1], "d10_r16": [1, 4] + [16] * 7 + [4, 1], "d6_r32": [1, 4, 16, 32, 16, 4, 1]}
    h = hashlib.sha256()
    for name, ranks in cases.items():
        base = train(rng, ranks)
        for mode, eps in ((0, 1e-10), (0, 1e-3), (1, 1e-3)):
            def once():
                tt = list(base)
                return T.tt_rank_reduce(tt, eps) if mode == 0 else T._tail_rank_reduce(tt, eps)
            out = once()
            if mode == 1:
                out, tail = out
                h.update(np.float64(tail if tail is not None else np.nan).tobytes())
            for c in out:
                h.update(D.read(c).tobytes())
            for _ in range(10):
                once()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                once()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / reps * 1e6
            print(f"{name:8s} mode {mode} eps {eps:g}: ranks {T.tt_ranks(out)}  {us:8.1f} us/call", flush=True)
    print("digest", h.hexdigest()[:16], flush=True)


if __name__ == "__main__":
    main()
