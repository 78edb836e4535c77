"""cProfile one run of the MI355X path; writes the top of the profile to gpurun_out/."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd._lib import lib  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg_name, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
max_it = int(sys.argv[5]) if len(sys.argv) > 5 else None
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", cfg_name + ".yaml")))


class Stop(Exception):
    pass


def cb(it):
    if max_it and it >= max_it:
        raise Stop


if os.environ.get("TTIPM_PROFILE_WARM", "1") == "1":  # plans, allocator and code pages first
    run_and_record(prob, cfg, seed, rank, verbose=False)
pr = cProfile.Profile()
l0 = lib.ttk_launch_count()
t = time.time()
pr.enable()
try:
    run_and_record(prob, cfg, seed, rank, verbose=False, iter_callback=cb)
except Stop:
    pass
pr.disable()
wall = time.time() - t
s = io.StringIO()
ps = pstats.Stats(pr, stream=s).sort_stats("tottime")
ps.print_stats(45)
ps.sort_stats("cumulative").print_stats(60)
ps.print_callers(r"\(read\)|\(dot\)|\(norm\)")
from ttipm_amd import dev as _D  # noqa: E402
ops = ""
if _D.OPSTATS is not None:
    for name, d in _D.OPSTATS.items():
        if name == "einsum_eq":
            ops += "EINSUM equations by calls:\n" + "".join(
                f"   {c[0]:8d}  {eq}\n" for eq, c in sorted(d.items(), key=lambda kv: -kv[1][0])[:30])
            continue
        tot = sum(v[1] for v in d.values())
        cnt = sum(v[0] for v in d.values())
        ops += f"OP {name}: {cnt} calls {tot:.3f}s\n"
        for shp, (c, t) in sorted(d.items(), key=lambda kv: -kv[1][1])[:25]:
            ops += f"   {str(shp):14s} {c:6d} {t * 1e3:9.2f}ms {t / c * 1e6:9.1f}us\n"
if _D.OPSTATS is not None and "svd" in _D.OPSTATS:
    bk = {}
    for (m, n), (c, t) in _D.OPSTATS["svd"].items():
        p_, q_ = min(m, n), max(m, n)
        key = next(f"p<={b}" for b in (4, 8, 16, 24, 32, 48, 64, 96, 128, 256, 10 ** 9) if p_ <= b)
        e = bk.setdefault(key, [0, 0.0, 0])
        e[0] += c
        e[1] += t
        e[2] = max(e[2], q_)
    ops += "SVD buckets (p=min dim): " + " | ".join(f"{k}: {v[0]} calls {v[1] * 1e3:.1f} ms (max q {v[2]})"
                                                   for k, v in bk.items()) + "\n"
out = f"wall {wall:.2f}s launches {lib.ttk_launch_count() - l0}\n" + ops + s.getvalue()
os.makedirs("gpurun_out", exist_ok=True)
open(f"gpurun_out/prof_{cfg_name}_s{seed}.txt", "w").write(out)
print(out[:3000])
