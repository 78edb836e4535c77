"""Aggregate kernel-dispatch rate of P processes (one stream each) launching tiny kernels back to
back (ttk_fill of one double): is the GPU's dispatch rate what bounds several solves in flight?
LR_KERNEL=eig / gemm: the same with one-workgroup eigensolves / multi-workgroup GEMMs (do the
processes' kernels run concurrently?); LR_HWQ: GPU_MAX_HW_QUEUES of the workers (default 8).
    python tools/launch_rate.py [launches_per_process] [P ...]"""
import os
import subprocess
import sys
import time


def worker(n):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    from ttipm_amd import dev as D
    from ttipm_amd._lib import lib
    import numpy as np
    z = D.empty(1)
    st = D._stream()
    kind = os.environ.get("LR_KERNEL", "fill")
    if kind == "fill":  # tiny launches: the dispatch rate
        def one():
            lib.ttk_fill(st, D._p(z), 1, 0.0)
    elif kind == "eig":  # one-workgroup ~0.45 ms kernels (syev_small n = 128): do processes overlap?
        M = np.random.default_rng(0).standard_normal((128, 128))
        A = D.from_numpy(M + M.T)
        wx = D.empty(int(lib.ttk_syev_extreme_work(128)))
        buf = D.empty(129)

        def one():
            lib.ttk_syev_extreme(st, D._p(A), 128, 0, D._p(buf), D._p(buf[1:]), D._p(wx))
    else:  # "gemm": multi-workgroup fp64 GEMMs (700 x 650 x 520)
        a = torch.randn(700, 520, dtype=torch.float64, device="cuda")
        b = torch.randn(520, 650, dtype=torch.float64, device="cuda")

        def one():
            D.matmul(a, b)
    for _ in range(20 if kind != "fill" else 200):
        one()
    torch.cuda.synchronize()
    print("ready", flush=True)
    sys.stdin.readline()
    t0 = time.perf_counter()
    for _ in range(n):
        one()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{t1 - t0} {t2 - t0}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        return worker(int(sys.argv[2]))
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    for P in [int(p) for p in (sys.argv[2:] or ["1", "2", "4", "8"])]:
        env = dict(os.environ, GPU_MAX_HW_QUEUES=os.environ.get("LR_HWQ", "8"))
        ps = [subprocess.Popen([sys.executable, __file__, "--worker", str(n)], stdin=subprocess.PIPE,
                               stdout=subprocess.PIPE, text=True, env=env) for _ in range(P)]
        for p in ps:
            while p.stdout.readline().strip() != "ready":
                pass
        t0 = time.perf_counter()
        for p in ps:
            p.stdin.write("go\n")
            p.stdin.flush()
        outs = [p.stdout.readline().split() for p in ps]
        wall = time.perf_counter() - t0
        for p in ps:
            p.wait()
        host = max(float(o[0]) for o in outs)
        print(f"P={P}: {P * n} launches in {wall:.3f} s -> {P * n / wall / 1e3:.0f} k launches/s "
              f"(per process {n / wall / 1e3:.0f} k/s; host enqueue {n / host / 1e3:.0f} k/s)", flush=True)


if __name__ == "__main__":
    main()
