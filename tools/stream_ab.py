"""Diagnostics (GPU): solves of maxcut_10 seeds on one GPU from ONE process, one solve per slot
thread (each its own created stream and libttk context, problems created before the threads start,
as bench.py's slots): per-solve s/IPM-iter per thread and the whole-job rate, against the same
seeds solved one at a time on the default stream.  Run it under different switches (e.g.
TTK_HOLD_GIL=1) to compare thread layouts.
    python tools/stream_ab.py [threads] [reps] [seeds, comma-separated]"""
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import yaml  # noqa: E402

from ttipm_amd import rng, shard  # noqa: E402
from ttipm_amd.utils import create, solve  # noqa: E402

nthr = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
seeds = [int(s) for s in (sys.argv[3] if len(sys.argv) > 3 else "41,235").split(",")]
if len(sys.argv) > 4:
    sys.setswitchinterval(float(sys.argv[4]))
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "maxcut_10.yaml")))
packed = {s: shard.pack(create("maxcut", cfg, s, 1, verbose=False)) for s in seeds}


def run(seed, n):
    out = []
    for _ in range(n):
        prep = shard.unpack(*packed[seed])
        t = time.perf_counter()
        r = solve(prep, cfg, quiet=True, verbose=False)
        torch.cuda.current_stream().synchronize()
        out.append(((time.perf_counter() - t), r["num_iters"], r["gap"]))
    return out


torch.cuda.set_device(0)
solo = {}
for s in seeds:
    run(s, 1)
    solo[s] = run(s, reps)
    print(f"solo seed {s}: s/iter {[round(w / i, 4) for w, i, _ in solo[s]]} gap {solo[s][0][2]!r}", flush=True)
res, ready = {}, threading.Barrier(nthr + 1)


def slot(j):
    torch.cuda.set_device(0)
    rng.private()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        sd = seeds[j % len(seeds)]
        run(sd, 1)
        ready.wait()
        res[j] = (sd, run(sd, reps))


th = [threading.Thread(target=slot, args=(j,)) for j in range(nthr)]
for t in th:
    t.start()
ready.wait()
t0 = time.perf_counter()
for t in th:
    t.join()
wall = time.perf_counter() - t0
its = 0
for j in range(nthr):
    sd, v = res[j]
    its += sum(i for _, i, _ in v)
    ok = all(g == solo[sd][0][2] for _, _, g in v)
    print(f"thread {j} seed {sd}: s/iter {[round(w / i, 4) for w, i, _ in v]} same gap as solo: {ok}", flush=True)
print(f"threads {nthr} hold_gil {os.environ.get('TTK_HOLD_GIL', '1')} switch {sys.getswitchinterval()}: "
      f"whole job {wall / its:.4f} s/IPM-iter ({its} iters in {wall:.2f} s)", flush=True)
