"""Seed-parallel multi-GPU execution -- SURVEY.md §8(e).

The reference runs its seed list serially (`src/utils.py:58-84`).  Seeds are independent solves, so
the MI355X path shards them: one process per GPU, GPU p takes seeds {s_i : i = p mod P}.

Collectives (RCCL over xGMI when the process group is "nccl", gloo on CPU):
  * ONE broadcast from rank 0 before any solve: rank 0 runs `create_problem` for every seed of the
    schedule and broadcasts the packed fp64 cores of (obj, L, bias, lag maps, mask) as a single
    device tensor, with the shapes and the NumPy MT19937 state after creation as a small object
    (the IPM's later random draws continue that stream, so each rank restores it before `tt_ipm`);
  * ONE all-gather of the per-seed result dicts after the loop.
There is no cross-GPU state inside the IPM loop."""
import numpy as np
import torch
import torch.distributed as dist

from . import dev as D
from .utils import create

_TT_KEYS = ("C", "L", "b", "mask")


def _tts(prep):
    out = [(k, prep[k]) for k in _TT_KEYS if prep[k] is not None]
    out += [("lag:" + k, prep["lag"][k]) for k in sorted(prep["lag"])]
    return out


def pack(prep):
    """(meta, flat) for one created problem; `flat` is one contiguous fp64 device tensor."""
    tts = _tts(prep)
    meta = {"seed": prep["seed"], "creation_time": prep["creation_time"],
            "rng_state": tuple(x.tolist() if isinstance(x, np.ndarray) else x for x in prep["rng_state"]),
            "tts": [(name, [tuple(c.shape) for c in tt]) for name, tt in tts]}
    flat = torch.cat([c.reshape(-1) for _, tt in tts for c in tt]) if tts else D.empty(0)
    return meta, flat


def unpack(meta, flat):
    """Inverse of `pack`; the cores are fresh contiguous device tensors (views are cloned)."""
    prep = {"seed": meta["seed"], "creation_time": meta["creation_time"], "mask": None, "lag": {}}
    name, keys, pos, has_gauss, cached = meta["rng_state"]
    prep["rng_state"] = (name, np.asarray(keys, dtype=np.uint32), pos, has_gauss, cached)
    o = 0
    for tname, shapes in meta["tts"]:
        cores = []
        for shp in shapes:
            n = int(np.prod(shp)) if len(shp) else 1
            cores.append(flat[o:o + n].clone().view(*shp))
            o += n
        if tname.startswith("lag:"):
            prep["lag"][tname[4:]] = cores
        else:
            prep[tname] = cores
    return prep


def broadcast_problems(problem, config, seeds, rank_tt, src=0):
    """Rank `src` creates every seed's problem; one broadcast delivers all of them to all ranks.
    Returns a list of (meta, flat) per seed (unpack with `unpack`, once per solve)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    me = dist.get_rank() if dist.is_initialized() else 0
    if me == src:
        packed = [pack(create(problem, config, s, rank_tt, verbose=False)) for s in seeds]
        metas = [m for m, _ in packed]
        sizes = [int(f.numel()) for _, f in packed]
        payload = torch.cat([f for _, f in packed]) if packed else D.empty(0)
    else:
        metas, sizes, payload = None, None, None
    if world > 1:
        obj = [metas, sizes]
        dist.broadcast_object_list(obj, src=src)
        metas, sizes = obj
        if me != src:
            payload = D.empty(sum(sizes))
        dist.broadcast(payload, src=src)
    out, o = [], 0
    for m, n in zip(metas, sizes):
        out.append((m, payload[o:o + n]))
        o += n
    return out


def my_seeds(seeds, rank, world):
    """Round-robin shard: rank p gets seeds[p::world]."""
    return list(seeds[rank::world])


def gather_results(results):
    """All-gather the per-rank lists of per-seed result dicts (flattened, rank order)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return list(results)
    buf = [None] * dist.get_world_size()
    dist.all_gather_object(buf, list(results))
    return [r for part in buf for r in part]


__all__ = ["pack", "unpack", "broadcast_problems", "my_seeds", "gather_results"]
