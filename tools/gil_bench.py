"""Host-side cost of tensor metadata calls, one thread and two threads of one process (CPU
tensors; runs anywhere): torch's own bindings (which release the GIL around each op) against the
GIL-holding helpers of _ttkbind (csrc/ttk_host_bind.cpp).
    python tools/gil_bench.py"""
import glob
import importlib.util
import os
import sys
import threading
import time

import torch

sys.setswitchinterval(0.0005)
N = 50000
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("_ttkbind", glob.glob(os.path.join(
    HERE, "tensor-train-interior-point-method_amd", "_ttkbind*.so"))[0])
B = importlib.util.module_from_spec(spec)
spec.loader.exec_module(B)


def run(fn, nthr):
    def work():
        for _ in range(N):
            fn()
    th = [threading.Thread(target=work) for _ in range(nthr)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    return (time.perf_counter() - t) / (N * nthr) * 1e6


a = torch.empty(4, 4, dtype=torch.float64)
b = torch.empty(16, dtype=torch.float64)
cases = {"torch.empty": lambda: torch.empty((4, 4), dtype=torch.float64), "bind.empty": lambda: B.empty(a, (4, 4)),
         "Tensor.view": lambda: b.view(4, 4), "bind.view": lambda: B.view(b, (4, 4)),
         "Tensor.t": lambda: a.t(), "bind.t": lambda: B.t(a),
         "Tensor.permute": lambda: a.permute(1, 0), "bind.permute": lambda: B.permute(a, (1, 0))}
for name, fn in cases.items():
    r1, r2 = run(fn, 1), run(fn, 2)
    print(f"{name:16s} 1 thread {r1:5.2f} us | 2 threads {r2:5.2f} us per call", flush=True)
