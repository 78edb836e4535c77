"""Restatement of opt_einsum 3.4.0's `contract_expression(eq, *shapes, optimize='greedy')` --
TEST INFRASTRUCTURE (oracle + golden-generation shim only).

The reference contracts every small tensor network through
`opt_einsum.contract_expression(equation, *shapes, optimize='greedy')` (`src/tt_ops.py:22-28`,
opt_einsum pinned at 3.4.0 by `env.yaml:10`).  opt_einsum is absent from this image, so its
published algorithm is restated here:

* path (`opt_einsum/paths.py::greedy` with `memory_limit=None`, i.e. `ssa_greedy_optimize` with the
  'memory-removed' cost = size(result) - size(a) - size(b), ties broken by SSA ids; dims shared by
  every operand are treated as output dims; identical index sets are Hadamard-merged first; leftover
  disconnected operands are joined by outer products smallest-first), converted with
  `ssa_to_linear`; one- and two-operand expressions take `[(0,)]` / `[(0, 1)]` directly
  (`opt_einsum/contract.py::contract_path`);
* execution (`opt_einsum/contract.py::_core_contract`): each pairwise step whose `blas.can_blas`
  test passes runs as `numpy.tensordot` over the removed indices followed by a transpose to the
  step's result order; any other step runs as a plain `numpy.einsum` (no path optimisation);
  intermediate index order is the "tensordot order" (`sorted(out_inds, key=all_input_inds.find)`);
* cost (`helpers.flop_count`): size of all indices in the step x max(1, terms - 1) (+1 when an
  index is summed) -- the FLOP convention of SURVEY.md §8(d).

NumPy's own `einsum_path(..., optimize='greedy')` is NOT a substitute: with its default memory cap
(the largest operand) it collapses the 4-operand local applies into one naive contraction
(~100x the FLOPs and a different rounding order).
"""
import heapq
import itertools
from collections import defaultdict
from functools import lru_cache

import numpy as np


def _size(key, sizes):
    n = 1
    for c in key:
        n *= sizes[c]
    return n


def _get_candidate(output, sizes, remaining, footprints, dim_ref_counts, k1, k2):
    either = k1 | k2
    two = k1 & k2
    one = either - two
    k12 = (either & output) | (two & dim_ref_counts[3]) | (one & dim_ref_counts[2])
    cost = _size(k12, sizes) - footprints[k1] - footprints[k2]  # 'memory-removed'
    id1, id2 = remaining[k1], remaining[k2]
    if id1 > id2:
        k1, id1, k2, id2 = k2, id2, k1, id1
    return (cost, id2, id1), k1, k2, k12


def _push_candidate(output, sizes, remaining, footprints, dim_ref_counts, k1, k2s, queue):
    cands = [_get_candidate(output, sizes, remaining, footprints, dim_ref_counts, k1, k2) for k2 in k2s]
    heapq.heappush(queue, min(cands, key=lambda c: c[0]))


def _update_ref_counts(dim_to_keys, dim_ref_counts, dims):
    for dim in dims:
        count = len(dim_to_keys[dim])
        if count <= 1:
            dim_ref_counts[2].discard(dim)
            dim_ref_counts[3].discard(dim)
        elif count == 2:
            dim_ref_counts[2].add(dim)
            dim_ref_counts[3].discard(dim)
        else:
            dim_ref_counts[2].add(dim)
            dim_ref_counts[3].add(dim)


def _ssa_greedy(inputs, output, sizes):
    if len(inputs) == 1:
        return [(0,)]
    inputs = [frozenset(x) for x in inputs]
    output = frozenset(output) | frozenset.intersection(*inputs)
    remaining = {}
    ssa_ids = itertools.count(len(inputs))
    ssa_path = []
    for ssa_id, key in enumerate(inputs):
        if key in remaining:
            ssa_path.append((remaining[key], ssa_id))
            remaining[key] = next(ssa_ids)
        else:
            remaining[key] = ssa_id
    dim_to_keys = defaultdict(set)
    for key in remaining:
        for dim in key - output:
            dim_to_keys[dim].add(key)
    dim_ref_counts = {cnt: set(dim for dim, keys in dim_to_keys.items() if len(keys) >= cnt) - output
                      for cnt in (2, 3)}
    footprints = {key: _size(key, sizes) for key in remaining}
    queue = []
    for dim, dim_keys in dim_to_keys.items():
        dim_keys = sorted(dim_keys, key=remaining.__getitem__)
        for i, k1 in enumerate(dim_keys[:-1]):
            _push_candidate(output, sizes, remaining, footprints, dim_ref_counts, k1, dim_keys[1 + i:], queue)
    while queue:
        _, k1, k2, k12 = heapq.heappop(queue)
        if k1 not in remaining or k2 not in remaining:
            continue  # obsolete candidate
        ssa_id1 = remaining.pop(k1)
        ssa_id2 = remaining.pop(k2)
        for dim in k1 - output:
            dim_to_keys[dim].remove(k1)
        for dim in k2 - output:
            dim_to_keys[dim].remove(k2)
        ssa_path.append((ssa_id1, ssa_id2))
        if k12 in remaining:
            ssa_path.append((remaining[k12], next(ssa_ids)))
        else:
            for dim in k12 - output:
                dim_to_keys[dim].add(k12)
        remaining[k12] = next(ssa_ids)
        _update_ref_counts(dim_to_keys, dim_ref_counts, k1 | k2 - output)  # precedence as published
        footprints[k12] = _size(k12, sizes)
        k1 = k12
        k2s = set(k2 for dim in k1 - output for k2 in dim_to_keys[dim])
        k2s.discard(k1)
        if k2s:
            _push_candidate(output, sizes, remaining, footprints, dim_ref_counts, k1, list(k2s), queue)
    queue = [(_size(key & output, sizes), ssa_id, key) for key, ssa_id in remaining.items()]
    heapq.heapify(queue)
    _, ssa_id1, k1 = heapq.heappop(queue)
    while queue:
        _, ssa_id2, k2 = heapq.heappop(queue)
        ssa_path.append((min(ssa_id1, ssa_id2), max(ssa_id1, ssa_id2)))
        k12 = (k1 | k2) & output
        ssa_id12 = next(ssa_ids)
        _, ssa_id1, k1 = heapq.heappushpop(queue, (_size(k12, sizes), ssa_id12, k12))
    return ssa_path


def _ssa_to_linear(ssa_path):
    ids = np.arange(1 + max(map(max, ssa_path)), dtype=np.int64)
    path = []
    for ssa in ssa_path:
        path.append(tuple(int(ids[s]) for s in ssa))
        for s in ssa:
            ids[s:] -= 1
    return path


def _can_blas(inputs, result, idx_removed, shapes):
    if len(inputs) != 2:
        return False
    left, right = inputs
    for c in set(left + right):
        nl, nr = left.count(c), right.count(c)
        if nl > 1 or nr > 1 or nl + nr > 2:
            return False
        if nl + nr - 1 == int(c in result):
            return False
    for c in idx_removed:
        if shapes[0][left.find(c)] != shapes[1][right.find(c)]:
            return False
    if len(idx_removed) == 0:
        return False
    sets = [set(x) for x in inputs]
    if inputs[0] == inputs[1]:
        return True  # DOT
    if sets[0] == sets[1]:
        return False
    keep_left, keep_right = sets[0] - idx_removed, sets[1] - idx_removed
    rs = len(idx_removed)
    if left[-rs:] == right[:rs] or left[:rs] == right[-rs:] or left[-rs:] == right[-rs:] or left[:rs] == right[:rs]:
        return True  # GEMM variants
    if len(keep_left) == 0 or len(keep_right) == 0:
        return False
    return True  # TDOT


@lru_cache(maxsize=8192)
def plan(eq, shapes):
    """(steps, flops): steps = [(positions, idx_removed, einsum_str, blas)] as opt_einsum builds them."""
    lhs, out = eq.replace(" ", "").split("->")
    terms = lhs.split(",")
    sizes = {}
    for t, sh in zip(terms, shapes):
        for c, n in zip(t, sh):
            if c in sizes and sizes[c] != 1 and n not in (1, sizes[c]):
                raise ValueError(f"einsum: index {c} has extents {sizes[c]} and {n}")
            if c not in sizes or sizes[c] == 1:
                sizes[c] = int(n)
    n_ops = len(terms)
    if n_ops == 1:
        path = [(0,)]
    elif n_ops == 2:
        path = [(0, 1)]
    else:
        path = _ssa_to_linear(_ssa_greedy(terms, out, sizes))
    input_sets = [frozenset(t) for t in terms]
    output_set = frozenset(out)
    ins, shps = list(terms), [tuple(s) for s in shapes]
    steps, flops = [], 0
    for cnum, inds in enumerate(path):
        inds = tuple(sorted(inds, reverse=True))
        contract = frozenset()
        remain_sets, idx_remain = [], set(output_set)
        for i, v in enumerate(input_sets):
            if i in inds:
                contract |= v
            else:
                remain_sets.append(v)
                idx_remain |= v
        new_result = frozenset(idx_remain) & contract
        idx_removed = contract - new_result
        remain_sets.append(new_result)
        input_sets = remain_sets
        op_factor = max(1, len(inds) - 1) + (1 if idx_removed else 0)
        flops += _size(contract, sizes) * op_factor
        tmp_in = [ins.pop(x) for x in inds]
        tmp_sh = [shps.pop(x) for x in inds]
        blas = _can_blas(tmp_in, new_result, idx_removed, tmp_sh)
        if cnum == len(path) - 1:
            res = out
        else:
            allin = "".join(tmp_in)
            res = "".join(sorted(new_result, key=allin.find))
        ins.append(res)
        shps.append(tuple(sizes[c] for c in res))
        steps.append((inds, idx_removed, ",".join(tmp_in) + "->" + res, blas))
    return steps, float(flops)


def flops(eq, shapes):
    return plan(eq, tuple(tuple(int(n) for n in s) for s in shapes))[1]


def contract(eq, *ops):
    """Evaluate as opt_einsum 3.4.0's compiled greedy expression does (numpy backend)."""
    steps, _ = plan(eq, tuple(tuple(o.shape) for o in ops))
    ops = list(ops)
    for inds, idx_rm, estr, blas in steps:
        tmp = [ops.pop(x) for x in inds]
        if blas:
            ins, res = estr.split("->")
            left, right = ins.split(",")
            tres = "".join(s for s in left + right if s not in idx_rm)
            lpos = tuple(left.find(s) for s in idx_rm)
            rpos = tuple(right.find(s) for s in idx_rm)
            view = np.tensordot(tmp[0], tmp[1], axes=(lpos, rpos))
            if tres != res:
                view = view.transpose(tuple(map(tres.index, res)))
        else:
            view = np.einsum(estr, *tmp)
        ops.append(view)
    return ops[0]
