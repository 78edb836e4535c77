"""Row a19 (step-size eigen-ALS) against the reference's own output: the device
`tt_max_generalised_eigen` (`src/tt_als.py:1132-1283`) and its two-site local solve
(`_step_size_local_solve`, :931-1038) on the calls recorded from the reference's IPM
(tests/golden/step.npz, tests/golden/make_step.py: maxcut_10 s14 assemblies 4-5, s41 assemblies 0-1).

Tolerances: step sizes 1e-12 relative (the device's dense eigenpairs against ARPACK's at tol 1e-8:
the step is a generalised eigenvalue, measured <= 4e-14); local output shapes (truncation rank + kick)
exactly except on the documented degenerate local eigenproblems (step_cases.DEVICE_RANK_DEPARTURES;
the oracle with exact eigensolves departs on exactly the same ones, tests/test_oracle_step.py)."""
import numpy as np
import pytest

from tests import step_cases as SC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ttipm_amd import _lib
    from ttipm_amd import dev as D
    assert _lib.lib is not None
    return D


def _up(D, tt):
    return None if tt is None else [D.from_numpy(c) for c in tt]


@pytest.mark.parametrize("case", SC.CASES)
def test_step_size_call_matches_reference(dev, case):
    from ttipm_amd import tt_eig as E
    D = dev
    A, Dl, x0, st, ref, xr = SC.call(case)
    np.random.set_state(st)
    l0 = D.lib.ttk_launch_count()
    s, x = E.tt_max_generalised_eigen(_up(D, A), _up(D, Dl), x0=_up(D, x0), tol=1e-8)
    assert D.lib.ttk_launch_count() > l0
    assert abs(s - ref) <= 1e-12 * ref, (s, ref)
    ranks, ref_ranks = [int(c.shape[-1]) for c in x], [c.shape[-1] for c in xr]
    if case not in SC.DEVICE_RANK_DEPARTURES:
        assert ranks == ref_ranks, (ranks, ref_ranks)
    else:
        print(case, "solution ranks", ranks, "reference", ref_ranks, "(degenerate local eigenproblems)")


@pytest.mark.parametrize("case", SC.CASES)
def test_step_size_local_solves_match_reference(dev, case):
    from ttipm_amd import tt_eig as E
    D = dev
    departures = set()
    for j in range(SC.nlocal(case)):
        args, bwd, st, exp = SC.local(case, j)
        np.random.set_state(st)
        dargs = [D.from_numpy(a) for a in args[:10]] + list(args[10:])
        s1, s2, step, res = E._step_size_local_solve(*dargs, bwd=bwd)
        assert abs(step - exp["step"]) <= 1e-12 * exp["step"], (j, step, exp["step"])
        if res is not None and not isinstance(res, E._Slot):
            r = float(D.read(res)) if hasattr(res, "shape") else float(res)
            assert abs(r - exp["res"]) <= 1e-6 * abs(exp["res"]) + 1e-12, (j, r, exp["res"])
        if (tuple(s1.shape), tuple(s2.shape)) != (exp["s1"].shape, exp["s2"].shape):
            departures.add(j)
            continue
        pd, pr = SC.product(D.read(s1), D.read(s2)), SC.product(exp["s1"], exp["s2"])
        dv = np.abs(np.sign(np.vdot(pd, pr)) * pd - pr).max() / np.abs(pr).max()
        assert dv <= 1.0, (j, dv)  # eigenvectors of the same eigenspace, sign-aligned
    assert departures == SC.DEVICE_RANK_DEPARTURES.get(case, set()), departures


@pytest.mark.parametrize("case", SC.CASES)
def test_native_eigen_als_bit_identical_to_python(dev, case):
    """_ttkbind.eig_als (csrc/ttk_host_eig.inc: the sweeps orchestrated in C++) against tt_eig.py's
    Python orchestration of the same libttk calls, from the same inputs and MT19937 state: the same
    step size, solution cores and random state afterwards, bit for bit, and the native path must
    actually have run (no silent rerun in Python)."""
    from ttipm_amd import tt_eig as E
    D = dev
    A, Dl, x0, st, ref, _ = SC.call(case)
    out = {}
    for native in (True, False):
        E._NATIVE = native
        try:
            np.random.set_state(st)
            n0 = E.NATIVE_CALLS["native"]
            s, x = E.tt_max_generalised_eigen(_up(D, A), _up(D, Dl), x0=_up(D, x0), tol=1e-8)
            ran = E.NATIVE_CALLS["native"] - n0
        finally:
            E._NATIVE = True
        out[native] = (s, [D.read(c) for c in x], np.random.get_state(), ran)
    (sn, xn, rn, ran_n), (sp, xp, rp, ran_p) = out[True], out[False]
    assert ran_n == 1 and ran_p == 0
    assert sn == sp, (sn, sp)
    assert [c.shape for c in xn] == [c.shape for c in xp]
    assert all(np.array_equal(a, b) for a, b in zip(xn, xp))
    assert np.array_equal(rn[1], rp[1]) and rn[2:] == rp[2:]


def test_step_size_chain_s14_assembly4(dev):
    """s14's assembly-4 step pairs as the IPM makes them: predictor (c16 x, c17 z), then the corrector
    (c18 x warm-started from c16's solution, c19 z from c17's), the MT19937 stream carried from c16's
    recorded state.  c16-c18 must equal the reference's step sizes; c19 is the departure of maxcut_10
    s14 (KNOWN_DEPARTURES): warm-started from the device's own c17 solution -- whose ranks differ on
    degenerate local eigenproblems -- the corrector's dual eigen-ALS settles at 0.5019 (the local
    optimum the reference also passes through: its first 12 local solves of c19 sit at 0.50189...),
    where the reference, warm-started from ARPACK's c17 solution, goes on to 0.4057."""
    from ttipm_amd import tt_eig as E
    D = dev
    np.random.set_state(SC.call("s14_c16")[3])
    xs, got = {}, {}
    for c, src in (("s14_c16", None), ("s14_c17", None), ("s14_c18", "s14_c16"), ("s14_c19", "s14_c17")):
        A, Dl, x0, _, ref, _ = SC.call(c)
        s, x = E.tt_max_generalised_eigen(_up(D, A), _up(D, Dl), x0=_up(D, x0) if src is None else xs[src], tol=1e-8)
        xs[c], got[c] = x, (s, ref)
    for c in ("s14_c16", "s14_c17", "s14_c18"):
        assert abs(got[c][0] - got[c][1]) <= 1e-12 * got[c][1], (c, got[c])
    s, ref = got["s14_c19"]
    if abs(s - ref) > 1e-8 * ref:
        assert abs(s - 0.5018947125927) <= 1e-9, s  # the documented other optimum, nothing else
        pytest.xfail(f"s14 c19 chained: {s:.10f} against the reference's {ref:.10f} (warm start from the device's "
                     "c17 eigenvectors on degenerate local eigenproblems; maxcut_10 s14 KNOWN_DEPARTURES)")


def test_native_eigen_als_slot_threads(dev):
    """Two solve threads of one process (bench.py's slot threads, the layout at N = 8: each with its own
    stream, libttk context and private MT19937) run the native eigen-ALS at the same time -- it releases
    the GIL for the whole call: every call's step, cores and random state equal the same call run alone
    on this thread, bit for bit, and every call ran natively."""
    import threading

    import torch

    from ttipm_amd import rng
    from ttipm_amd import tt_eig as E
    D = dev
    cases = [c for c in SC.CASES if c.startswith("s41")][:4]

    def run(c, R):
        A, Dl, x0, st, _, _ = SC.call(c)
        R.set_state(st)
        s, x = E.tt_max_generalised_eigen(_up(D, A), _up(D, Dl), x0=_up(D, x0), tol=1e-8)
        return s, [D.read(t) for t in x], R.get_state()

    n0 = E.NATIVE_CALLS["native"]
    ref = {c: run(c, np.random.mtrand._rand) for c in cases}
    out, errs = {}, []

    def work(mine):
        try:
            torch.cuda.set_stream(torch.cuda.Stream())
            R = rng.private()
            for c in mine:
                out[c] = run(c, R)
            torch.cuda.current_stream().synchronize()
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append(e)

    threads = [threading.Thread(target=work, args=(cases[i::2],)) for i in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not errs, errs
    assert E.NATIVE_CALLS["native"] - n0 == 2 * len(cases)
    for c in cases:
        (s0, x0, r0), (s1, x1, r1) = ref[c], out[c]
        assert s0 == s1, (c, s0, s1)
        assert all(np.array_equal(a, b) for a, b in zip(x0, x1)), c
        assert np.array_equal(r0[1], r1[1]) and r0[2:] == r1[2:], c
    D.check_handoffs()
