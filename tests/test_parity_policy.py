"""The whole-solve parity policy's end-point rules (tests/parity_policy.py) on the reference's own runs
(tests/golden/runs.json), CPU only: what they accept and what they reject (a
pathological end point is bounded by the pathological runs it claims to match; VERDICT r5 item 2: a
key with a single converged unmodified run gets a rule fixed before the device runs)."""
import copy

import pytest

from tests import parity_policy as PP


def _end(**kw):
    return {"num_iters": kw.get("num_iters"), "gap": kw.get("gap"), "feas": kw.get("feas")}


def test_unmodified_runs_pass_their_own_end_point_rule():
    """every full-solve key whose unmodified runs branch: each of those runs passes check_end_point
    (the rule admits the reference itself)"""
    keys = [k for k, v in PP.RUNS.items() if not v.get("bounded") and not any(k.endswith(x) for x in PP.ALL_TWINS)
            and any(k + x in PP.RUNS for x in PP.NOISE_TWINS) and not k.endswith("_shipped")]
    assert keys
    for k in keys:
        for r in PP.unmodified_runs(k):
            PP.check_end_point(k, r)


def test_pathological_end_point_is_bounded_by_the_pathological_runs():
    k = "maxcut_12_r2_s45"  # golden 21 iterations, _h1 29, both pathological (gap 2.9e-3, 3.0e-3)
    PP.check_end_point(k, _end(num_iters=22, gap=3.1e-3, feas=7.1e-9))  # the device's r06 end point
    for bad in (_end(num_iters=12, gap=3.1e-3, feas=7.1e-9),   # stalls at another iteration count
                _end(num_iters=22, gap=5.0, feas=7.1e-9),      # another magnitude
                _end(num_iters=22, gap=float("nan"), feas=7.1e-9)):
        with pytest.raises(AssertionError):
            PP.check_end_point(k, bad)
    with pytest.raises(AssertionError):  # s41's unmodified runs all converge: no pathological basin
        PP.check_end_point("maxcut_10_r1_s41", _end(num_iters=9, gap=2e-3, feas=1e-9))


def test_single_converged_run_rule():
    """maxcut_12 s53: golden, _h1, _h3 end pathological, _h2 converges (29 iterations, gap 4.0e-4):
    a converged end point must lie in _h2's relaxed box"""
    k = "maxcut_12_r2_s53"
    good = [r for r in PP.unmodified_runs(k) if not PP.is_pathological(r)]
    assert len(good) == 1
    PP.check_end_point(k, _end(num_iters=29, gap=5.6e-4, feas=5.1e-9))  # the device's r06 end point
    for bad in (_end(num_iters=20, gap=5.6e-4, feas=5.1e-9), _end(num_iters=29, gap=5e-5, feas=5.1e-9),
                _end(num_iters=29, gap=5.6e-4, feas=1e-6)):
        with pytest.raises(AssertionError):
            PP.check_end_point(k, bad)


def test_maxcut_12_s1_device_end_point_is_rejected():
    """extra seed 1: the golden converges after 16 iterations, _h3 ends pathological after 11 (gap
    9.4); the device's end point (29 iterations, gap 1.9e-2) lands in neither basin -- rejected (it
    passed silently under round 5's rule), hence its KNOWN_EXTRA_DEPARTURES entry"""
    with pytest.raises(AssertionError):
        PP.check_end_point("maxcut_12_r2_s1", _end(num_iters=29, gap=1.949e-2, feas=1.19e-5))
    assert "maxcut_12_r2_s1" in PP.KNOWN_EXTRA_DEPARTURES


def test_extra_follow_floor():
    """check_extra_follow_floor: a trace equal to the followed unmodified run passes, one that leaves
    it early fails, a non-finite end point fails"""
    k = "maxcut_12_r2_s1"
    t = copy.deepcopy(PP.RUNS[k + "_h3"]["trace"])
    end = _end(num_iters=29, gap=1.9e-2, feas=1.2e-5)
    PP.check_extra_follow_floor(k, t, end)
    off = copy.deepcopy(t)
    off[1]["mu"] *= 1.01
    with pytest.raises(AssertionError):
        PP.check_extra_follow_floor(k, off, end)
    with pytest.raises(AssertionError):
        PP.check_extra_follow_floor(k, t, _end(num_iters=29, gap=float("inf"), feas=1e-5))


def test_envelope_only_is_capped():
    """ENVELOPE_ONLY (the follow rule against a diagnostic twin instead of an unmodified run) stays a
    one-key exception, and its key still has to land in the unmodified envelope"""
    assert set(PP.ENVELOPE_ONLY) == {"maxcut_10_r1_s23"}
