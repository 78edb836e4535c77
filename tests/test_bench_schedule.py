"""bench.py's seed schedule: YAML seeds only, shard dealing across ranks and
solves in flight, maxcut_12 r=2 (configs[4]) on 8 GPUs with the vetted extra seeds."""
import json
import os
import sys

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _cfg(name):
    return yaml.safe_load(open(os.path.join(ROOT, "configs", name)))


def test_maxcut10_single_gpu_uses_yaml_seeds_only():
    cfg = _cfg("maxcut_10.yaml")
    for P in (1, 2, 4):
        seeds, sched, slots = bench.make_schedule(cfg, "maxcut_10.yaml", None, 5, 1, 0, P, "shard")
        assert seeds == cfg["seeds"]
        assert all(len(st) == P for st in sched)
        assert {s for st in sched for s in st} == set(cfg["seeds"])
        assert [[st[j] for st in sched] for j in range(P)] == slots


def test_maxcut12_eight_ranks_distinct_seeds_per_step():
    cfg = _cfg("maxcut_12.yaml")
    per_rank = []
    for rank in range(8):
        seeds, sched, slots = bench.make_schedule(cfg, "maxcut_12.yaml", None, 2, 8, rank, 1, "shard")
        assert len(seeds) == 8 and seeds[:5] == cfg["seeds"] and seeds[5:] == bench.EXTRA_SEEDS["maxcut_12.yaml"]
        per_rank.append(slots[0])
    for i in range(2):  # each step: the 8 ranks solve the 8 distinct seeds
        assert sorted(r[i] for r in per_rank) == sorted(seeds)
    # with two solves in flight per GPU every seed is solved exactly twice per step
    _, sched, _ = bench.make_schedule(cfg, "maxcut_12.yaml", None, 1, 8, 0, 2, "shard")
    assert sorted(sched[0]) == sorted(seeds * 2)


def test_extra_seeds_are_vetted_by_reference_runs():
    """The extra seeds are non-pathological in the reference's own runs (src/utils.py:67-84)."""
    runs = json.load(open(os.path.join(ROOT, "tests", "golden", "runs.json")))
    for s in bench.EXTRA_SEEDS["maxcut_12.yaml"]:
        if f"maxcut_12_r2_s{s}" not in runs:
            pytest.skip(f"reference run maxcut_12_r2_s{s} not in runs.json")
        r = runs[f"maxcut_12_r2_s{s}"]
        assert r["num_iters"] is not None and r["gap"] <= 1e-3 and r["feas"] <= 1e-3, (s, r["gap"], r["feas"])


def test_replica_schedule():
    cfg = _cfg("maxcut_10.yaml")
    _, sched, _ = bench.make_schedule(cfg, "maxcut_10.yaml", None, 3, 2, 1, 1, "replica")
    assert sched == [[41, 41], [23, 23], [235, 235]]


def test_default_inflight_caps_processes_per_node():
    """4 solves in flight per GPU up to 4 GPUs, and a node never runs more than 16 solve processes
    (DEFAULT_THREADS slot threads per process)."""
    assert [bench.default_inflight(w) for w in (1, 2, 4, 8)] == [4, 4, 4, 2]
    T = bench.DEFAULT_THREADS
    assert all(w * -(-bench.default_inflight(w) // T) <= 16 for w in (1, 2, 4, 8, 16))
