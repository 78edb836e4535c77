"""Seed sharding across ranks with the gloo backend, world_size 2, on CPU:
rank 0 creates both problems, one broadcast delivers them, each rank solves its own seed through
the product host path (libttk emulated), results are all-gathered and match the reference.
This checks the sharding plumbing (broadcast, schedule, all-gather) on CPU; the gap tolerance (1e-4)
is the emulated library's, not a parity claim -- the device's end points under sharding are
checked on hardware by the 2-rank rehearsal (profiles/r06_rehearsal_maxcut10_n2_gloo_detail.json:
every seed ends on its N = 1 result to the last digit)."""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from tests.emu_ttk import emulated_ttipm
    emulated_ttipm()
    import torch.distributed as dist
    import yaml
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ttipm_amd import shard
    from ttipm_amd.utils import create, solve
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "maxcut_5.yaml")))
    seeds = [0, 319]
    packed = shard.broadcast_problems("maxcut", cfg, seeds, 1)
    mine = shard.my_seeds(list(range(len(seeds))), rank, world)
    res = []
    for i in mine:
        prep = shard.unpack(*packed[i])
        local = create("maxcut", cfg, seeds[i], 1, verbose=False)  # what this rank would build itself
        same = all(bool((a == b).all()) for a, b in zip(prep["L"], local["L"])) and \
            all(bool((a == b).all()) for a, b in zip(prep["C"], local["C"]))
        r = solve(prep, cfg, quiet=True, verbose=False)
        res.append({"seed": r["seed"], "gap": r["gap"], "num_iters": r["num_iters"], "same_problem": same,
                    "rank": rank})
    allres = shard.gather_results(res)
    if rank == 0:
        json.dump(allres, open(out, "w"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_two_rank_seed_sharding(tmp_path):
    out = str(tmp_path / "res.json")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    res = {r["seed"]: r for r in json.load(open(out))}
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "runs.json")))
    assert set(res) == {0, 319}
    assert res[0]["rank"] == 0 and res[319]["rank"] == 1
    for seed in (0, 319):
        g = gold[f"maxcut_5_r1_s{seed}"]
        assert res[seed]["same_problem"]
        assert res[seed]["num_iters"] == g["num_iters"]
        assert abs(res[seed]["gap"] - g["gap"]) <= 1e-4 * g["gap"]
