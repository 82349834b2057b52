"""The IPC transport's protocol (csrc/comm/ipc.h) on the host: one thread per rank.

Each rank pulls its receives out of the senders' windows between flag barriers, and collectives
(builtin / rsag / hier_coll) are emulated by pulls and k-way reduces -- the same schedule matching
and barrier sequence the GPU transport launches (ipc_sync.hip + the multi-lane copy / reduce
kernels). Checked against the fp64 mean with rank-distinct inputs and odd sizes, like the
virtual-rank tests of the RCCL schedules (tests/test_comm_plans.py); results must be bitwise
identical on every rank. Reference schedules: /root/reference/src/allreduce.py:9-170,
/root/reference/src/reducers.py:38-69.
"""
import pytest
import torch

from distributed_learning_amd.ops import _ext
from distributed_learning_amd.parallel.virtual import ipc_host_allreduce, virtual_allreduce

pytestmark = pytest.mark.skipif(not _ext.available(), reason="native extension not built")

FLAT = ["builtin", "ring", "direct", "central", "rsag", "ring_pipe"]
HIER = ["hier_ring", "hier_coll", "hier_central"]


def _inputs(N, n, dtype, seed=0):
    g = torch.Generator().manual_seed(seed * 7919 + n * 31 + N)
    return [(torch.randn(n, generator=g) * (1 + r)).to(dtype) for r in range(N)]


def _check(bufs, xs, tol_rel):
    ref = torch.stack([x.double() for x in xs]).mean(0)
    for b in bufs[1:]:
        assert torch.equal(bufs[0], b), "ranks disagree after the all-reduce"
    err = (bufs[0].double() - ref).abs()
    bound = tol_rel * (torch.stack([x.double().abs() for x in xs]).sum(0) / len(xs) + 1e-30)
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("N", [2, 3, 4, 8])
@pytest.mark.parametrize("algo", FLAT)
def test_ipc_flat_fp32(N, algo):
    for n in [1, 7, 63, 64 * N - 1, 1000, 50_003]:
        for ch in ([1, 3, 7] if algo in ("ring", "ring_pipe") else [0]):
            xs = _inputs(N, n, torch.float32)
            bufs = [x.clone() for x in xs]
            ipc_host_allreduce(bufs, algo, channels=ch)
            _check(bufs, xs, 1e-5 * N)


@pytest.mark.parametrize("N,L", [(4, 2), (8, 4), (8, 2), (6, 3), (4, 1)])
@pytest.mark.parametrize("algo", HIER)
def test_ipc_hierarchical_fp32(N, L, algo):
    for n in [1, 5, 64 * N + 3, 4099, 20_001]:
        xs = _inputs(N, n, torch.float32)
        bufs = [x.clone() for x in xs]
        ipc_host_allreduce(bufs, algo, local_size=L, channels=3)
        _check(bufs, xs, 1e-5 * N)


@pytest.mark.parametrize("algo", ["ring", "direct", "builtin", "hier_coll"])
def test_ipc_matches_virtual_ranks_bitwise(algo):
    """Same plans, same per-element summation order where the schedule fixes it: the IPC pulls give
    exactly the virtual-rank (copy-link) result for the P2P schedules."""
    N, n = 4, 12_345
    xs = _inputs(N, n, torch.float32, seed=5)
    a = [x.clone() for x in xs]
    b = [x.clone() for x in xs]
    ls = 2 if algo.startswith("hier") else None
    ipc_host_allreduce(a, algo, local_size=ls)
    virtual_allreduce(b, algo, local_size=ls)
    if algo in ("ring", "direct"):
        for u, v in zip(a, b):
            assert torch.equal(u, v)
    else:  # emulated collectives sum in member order in both executors
        for u, v in zip(a, b):
            torch.testing.assert_close(u, v, rtol=1e-6, atol=1e-6)


def test_ipc_bf16_fp32_accumulation():
    N, n = 8, 20_011
    xs = _inputs(N, n, torch.bfloat16, seed=3)
    ref = torch.stack([x.double() for x in xs]).mean(0)
    acc = [x.clone() for x in xs]
    ipc_host_allreduce(acc, "direct", accum_fp32=True)
    half_ulp = torch.clamp(ref.abs(), min=1e-30) * 2.0 ** -8
    assert bool(((acc[0].double() - ref).abs() <= half_ulp * 1.001 + 1e-6).all())
    for b in acc[1:]:
        assert torch.equal(acc[0], b)


def test_ipc_sum_and_channel_codes():
    N, n = 4, 4096
    xs = _inputs(N, n, torch.float32, seed=9)
    bufs = [x.clone() for x in xs]
    ipc_host_allreduce(bufs, "ring:2", average=False)
    ref = torch.stack([x.double() for x in xs]).sum(0)
    assert float((bufs[0].double() - ref).abs().max()) < 1e-4
