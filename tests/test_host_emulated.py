"""Product HOST logic (einsum planner, TT algebra, AMEn sweeps, LGMRES bookkeeping, IPM control
flow) on CPU, with the libttk C ABI replaced by the NumPy emulator in tests/emu_ttk.py.  The GPU
run of the same path is tests/test_gpu_parity.py; this file checks the host side alone against
the reference golden runs."""
import json
import os

import pytest
import yaml

from tests.emu_ttk import emulated_ttipm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "runs.json")))


@pytest.fixture(scope="module")
def pkg():
    return emulated_ttipm()


def test_maxcut_5_seed0_matches_reference(pkg):
    from ttipm_amd.utils import run_and_record
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "maxcut_5.yaml")))
    trace = []
    r = run_and_record("maxcut", cfg, 0, 1, trace=trace, verbose=False)
    g = GOLD["maxcut_5_r1_s0"]
    assert r["num_iters"] == g["num_iters"]
    assert r["ranksX"] == g["ranksX"] and r["ranksZ"] == g["ranksZ"]
    assert r["gap"] == pytest.approx(g["gap"], rel=1e-4)
    assert r["feas"] == pytest.approx(g["feas"], rel=1e-3)
    for a, b in zip(trace, g["trace"]):
        assert a["ranksX"] == b["ranksX"]
        assert a["mu"] == pytest.approx(b["mu"], rel=1e-4)


def test_shard_pack_roundtrip(pkg):
    import numpy as np
    from ttipm_amd import shard
    from ttipm_amd.utils import create
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "maxcut_5.yaml")))
    prep = create("maxcut", cfg, 319, 1, verbose=False)
    meta, flat = shard.pack(prep)
    back = shard.unpack(meta, flat)
    for k in ("C", "L", "b"):
        assert len(back[k]) == len(prep[k])
        for a, b in zip(back[k], prep[k]):
            assert tuple(a.shape) == tuple(b.shape) and bool((a == b).all())
    for k in prep["lag"]:
        for a, b in zip(back["lag"][k], prep["lag"][k]):
            assert bool((a == b).all())
    s0, s1 = prep["rng_state"], back["rng_state"]
    assert s0[0] == s1[0] and np.array_equal(s0[1], s1[1]) and s0[2:] == s1[2:]
