"""The device step-size eigen-ALS on the reference's own recorded calls (tests/golden/step.npz).

    python tools/step_fixture_dev.py [CASE ...] [--local]

Per call: the reference's step and solution ranks next to the device's on the same inputs and MT19937
state.  --local: every recorded two-site local solve replayed on its own (the reference's inputs,
RNG state and step), step in / out and output core shapes against the reference's."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd import tt_eig as E  # noqa: E402

F = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "step.npz"))
LOCAL_ARGS = ("p1", "p2", "XAX_k", "A_k", "A_kp1", "XAX_k2", "XDX_k", "D_k", "D_kp1", "XDX_k2", "step",
              "size_limit", "trunc_tol", "eps", "max_rank", "bwd")


def tt(name, up=True):
    if name + "/n" not in F:
        return None
    cores = [F[f"{name}/{i}"].copy() for i in range(int(F[name + "/n"]))]
    return [D.from_numpy(c) for c in cores] if up else cores


def set_rng(p):
    np.random.set_state(("MT19937", F[p + "/key"], int(F[p + "/pos"]), int(F[p + "/g"]), float(F[p + "/c"])))


def run_call(c):
    set_rng(c + "/rng")
    s, x = E.tt_max_generalised_eigen(tt(c + "/A"), tt(c + "/Delta"), x0=tt(c + "/x0"), tol=1e-8)
    ref = float(F[c + "/step"])
    rr = [a.shape[-1] for a in tt(c + "/x", False)][:-1]
    dr = [int(a.shape[-1]) for a in x][:-1]
    print(f"{c}: ref {ref:.12e} dev {s:.12e} rel {abs(s - ref) / ref:.2e} ranks ref {rr} dev {dr}", flush=True)
    return s, ref


def run_local(c):
    n = int(F[c + "/nlocal"])
    for j in range(n):
        p = f"{c}/l{j}"
        a = [F[f"{p}/{k}"] for k in LOCAL_ARGS]
        args = [D.from_numpy(np.array(v)) for v in a[:10]] + [float(a[10]), int(a[11]), float(a[12]), float(a[13]),
                                                                int(a[14])]
        set_rng(p + "/rng")
        s1, s2, step, res = E._step_size_local_solve(*args, bwd=bool(a[15]))
        ref = float(F[p + "/step_out"])
        rs = (F[p + "/s1"].shape, F[p + "/s2"].shape)
        ds = (tuple(s1.shape), tuple(s2.shape))
        prod_d = np.einsum("rny,ytR->rntR", D.read(s1), D.read(s2))
        prod_r = np.einsum("rny,ytR->rntR", F[p + "/s1"], F[p + "/s2"])
        if prod_d.shape == prod_r.shape:
            sg = np.sign(np.vdot(prod_d, prod_r)) or 1.0
            dv = np.abs(sg * prod_d - prod_r).max() / max(np.abs(prod_r).max(), 1e-300)
        else:
            dv = np.nan
        print(f"  l{j} m={int(np.prod(prod_r.shape))} bwd={bool(a[15])} step {float(a[10]):.12e} -> ref {ref:.12e} "
              f"dev {step:.12e} rel {abs(step - ref) / ref:.1e} shapes {'==' if rs == ds else f'ref {rs} dev {ds}'} "
              f"sol {dv:.1e}", flush=True)


def run_chain():
    """s14's assembly-4 step pairs as the IPM makes them: c18 warm-started from c16's solution, c19
    from c17's (`status.eigen_x0 / eigen_z0`), the RNG stream carried from c16's recorded state"""
    set_rng("s14_c16/rng")
    xs = {}
    for c, src in (("s14_c16", None), ("s14_c17", None), ("s14_c18", "s14_c16"), ("s14_c19", "s14_c17")):
        x0 = tt(c + "/x0") if src is None else xs[src]
        s, x = E.tt_max_generalised_eigen(tt(c + "/A"), tt(c + "/Delta"), x0=x0, tol=1e-8)
        xs[c] = x
        print(f"chain {c}: ref {float(F[c + '/step']):.12e} dev {s:.12e} ranks {[int(a.shape[-1]) for a in x][:-1]}",
              flush=True)


if __name__ == "__main__":
    if "--chain" in sys.argv:
        run_chain()
        sys.exit(0)
    cases = [a for a in sys.argv[1:] if not a.startswith("--")] or [str(c) for c in F["cases"]]
    for c in cases:
        run_call(c)
        if "--local" in sys.argv:
            run_local(c)
