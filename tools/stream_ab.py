"""Diagnostics (GPU): one seed's solve on the process's default stream, then on a created stream,
then two slot threads each on its own created stream -- per-solve s/IPM-iter for each layout.
    python tools/stream_ab.py [seed] [reps]"""
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import yaml  # noqa: E402

from ttipm_amd import rng  # noqa: E402
from ttipm_amd.utils import create, solve  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 41
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
flags = os.environ.get("TTIPM_AB_FLAGS", "")
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "maxcut_10.yaml")))


def run(n):
    out = []
    for _ in range(n):
        prep = create("maxcut", cfg, seed, 1, verbose=False)
        t = time.perf_counter()
        r = solve(prep, cfg, quiet=True, verbose=False)
        torch.cuda.current_stream().synchronize()
        out.append((time.perf_counter() - t) / r["num_iters"])
    return out


def show(tag, v):
    print(f"{tag:28s} median {statistics.median(v):.4f}  {['%.4f' % x for x in v]}", flush=True)


torch.cuda.set_device(0)
run(1)
show("default stream", run(reps))
if "high" in flags:
    s = torch.cuda.Stream(priority=-1)
elif "ext" in flags:
    import ctypes
    h = ctypes.c_void_p()
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0  # hipStreamNonBlocking
    s = torch.cuda.ExternalStream(h.value)
else:
    s = torch.cuda.Stream()
with torch.cuda.stream(s):
    run(1)
    show("created stream", run(reps))
res = {}


def slot(j):
    torch.cuda.set_device(0)
    rng.private()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        run(1)
        res[j] = run(reps)


th = [threading.Thread(target=slot, args=(j,)) for j in range(2)]
t0 = time.perf_counter()
for t in th:
    t.start()
for t in th:
    t.join()
for j in range(2):
    show(f"thread {j} (2 in flight)", res[j])
print("wall", time.perf_counter() - t0)
