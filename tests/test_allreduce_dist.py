"""All-reduce algorithms vs ``dist.all_reduce`` on Gloo ranks (SURVEY.md §7.4 tests/dist).

Rank-distinct data; sizes include numel < N and numel % N != 0 (the reference's padding branch,
allreduce.py:59-60); multi-channel rings; the 2-step hierarchical reducer on virtual nodes.
"""
import pytest
import torch
import torch.distributed as dist

from dist_util import run
from distributed_learning_amd.parallel.allreduce import (ALGORITHMS, edge_disjoint_rings, get_algorithm,
                                                         split_ranges)

SIZES = [1, 2, 3, 7, 64, 65, 1000, 4097, 100_003]


def _algos(rank, world, sizes, algos, channels_list):
    out = {}
    for n in sizes:
        base = torch.arange(n, dtype=torch.float64) * 1e-3
        x = base + rank * 1.5 + torch.sin(base * (rank + 1))
        ref = x.clone()
        dist.all_reduce(ref)
        ref /= world
        for a in algos:
            for ch in channels_list if a.startswith("ring") else [1]:
                y = x.clone()
                get_algorithm(a, ch)(y)
                out[(a, ch, n)] = float((y - ref).abs().max())
    return out


@pytest.mark.parametrize("world", [2, 3, 4])
def test_algorithms_match_builtin(world):
    res = run(_algos, world, SIZES, sorted(ALGORITHMS), [1, 2, 3])
    for r in res:
        for k, err in r.items():
            assert err < 1e-9, (k, err)


def _hier(rank, world, local_size, algo, sizes):
    from distributed_learning_amd.parallel.reducers import HierarchicalReducer

    red = HierarchicalReducer(local_size, algo)
    out = {}
    for n in sizes:
        x = torch.randn(n, dtype=torch.float64, generator=torch.Generator().manual_seed(rank * 100 + n))
        ref = x.clone()
        dist.all_reduce(ref)
        ref /= world
        red.reduce(x)
        out[n] = float((x - ref).abs().max())
    return out


@pytest.mark.parametrize("local_size,algo", [(2, "ring"), (2, "central"), (1, "ring"), (4, "ring")])
def test_hierarchical_reducer(local_size, algo):
    res = run(_hier, 4, local_size, algo, [1, 5, 1000, 4099])
    for r in res:
        assert max(r.values()) < 1e-9, r


def test_edge_disjoint_rings_cover_all_links():
    rings = edge_disjoint_rings(8, 7)
    assert len(rings) == 7
    edges = set()
    for r in rings:
        assert sorted(r) == list(range(8))
        e = {(r[i], r[(i + 1) % 8]) for i in range(8)}
        assert not (e & edges)
        edges |= e
    assert len(edges) == 56  # every directed xGMI link of an 8-GPU node, exactly once
    assert len(edge_disjoint_rings(2, 7)) == 1
    assert len(edge_disjoint_rings(4, 3)) >= 2


def test_split_ranges():
    for n in [0, 1, 5, 63, 64, 65, 1000, 100_001]:
        for parts in [1, 2, 3, 7, 8]:
            r = split_ranges(n, parts)
            assert len(r) == parts
            assert sum(l for _, l in r) == n
            pos = 0
            for off, ln in r:
                if ln:
                    assert off == pos
                    pos += ln
