"""The C++ collective schedules (csrc/comm/plan.cpp) executed for N virtual ranks on the CPU.

``virtual_allreduce`` runs exactly the Plans the RCCL engine replays on a multi-GPU node (chunk
geometry, edge-disjoint channel rings, reduce arithmetic, fp32 staging of bf16 buckets) in
lockstep, matching every send with its receive — so the N>1 paths of every algorithm are checked
here without GPUs (the GPU twin is tests/test_gpu_engine_vranks.py). Reference schedules:
/root/reference/src/allreduce.py:9-170, /root/reference/src/reducers.py:38-69.
"""
import re

import pytest
import torch

from distributed_learning_amd.ops import _ext
from distributed_learning_amd.parallel.allreduce import split_ranges
from distributed_learning_amd.parallel.virtual import plan_text, virtual_allreduce

pytestmark = pytest.mark.skipif(not _ext.available(), reason="native extension not built")

FLAT = ["builtin", "ring", "direct", "central", "rsag", "ring_pipe"]
HIER = ["hier_ring", "hier_coll", "hier_central"]


def _inputs(N, n, dtype, seed=0):
    g = torch.Generator().manual_seed(seed * 7919 + n * 31 + N)
    return [(torch.randn(n, generator=g) * (1 + r)).to(dtype) for r in range(N)]


def _check(bufs, xs, tol_rel):
    ref = torch.stack([x.double() for x in xs]).mean(0)
    for b in bufs[1:]:
        assert torch.equal(bufs[0], b), "virtual ranks disagree after the all-reduce"
    err = (bufs[0].double() - ref).abs()
    bound = tol_rel * (torch.stack([x.double().abs() for x in xs]).sum(0) / len(xs) + 1e-30)
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("N", [2, 3, 4, 8])
@pytest.mark.parametrize("algo", FLAT)
def test_flat_algorithms_fp32(N, algo):
    for n in [1, 7, 63, 64 * N - 1, 1000, 100_003]:
        for ch in ([1, 3, 7] if algo in ("ring", "ring_pipe") else [0]):
            xs = _inputs(N, n, torch.float32)
            bufs = [x.clone() for x in xs]
            virtual_allreduce(bufs, algo, channels=ch)
            _check(bufs, xs, 1e-5 * N)


@pytest.mark.parametrize("N,L", [(4, 2), (8, 4), (8, 2), (6, 3), (4, 1), (4, 4)])
@pytest.mark.parametrize("algo", HIER)
def test_hierarchical_fp32(N, L, algo):
    for n in [1, 5, 63, 64 * N + 3, 4099, 50_001]:
        xs = _inputs(N, n, torch.float32)
        bufs = [x.clone() for x in xs]
        virtual_allreduce(bufs, algo, local_size=L, channels=3)
        _check(bufs, xs, 1e-5 * N)


@pytest.mark.parametrize("algo", ["ring", "direct", "central", "hier_ring", "builtin"])
def test_bf16_and_fp32_accumulation(algo):
    N, n = 8, 20_011
    xs = _inputs(N, n, torch.bfloat16, seed=3)
    ref = torch.stack([x.double() for x in xs]).mean(0)
    plain = [x.clone() for x in xs]
    virtual_allreduce(plain, algo, local_size=4 if algo.startswith("hier") else None)
    acc = [x.clone() for x in xs]
    virtual_allreduce(acc, algo, local_size=4 if algo.startswith("hier") else None, accum_fp32=True)
    # fp32 staging: one rounding to bf16 at the end -> within half a bf16 ulp (+fp32 noise)
    exact = ref.to(torch.bfloat16).double()
    half_ulp = torch.clamp(ref.abs(), min=1e-30) * 2.0 ** -8  # bf16: 8 significant bits
    assert bool(((acc[0].double() - ref).abs() <= half_ulp * 1.001 + 1e-6).all())
    assert float((acc[0].double() - exact).abs().max()) <= float(2 * half_ulp.max())
    e_plain = float((plain[0].double() - ref).abs().mean())
    e_acc = float((acc[0].double() - ref).abs().mean())
    assert e_acc <= e_plain  # bf16 partial sums on the wire round at every step
    for b in acc[1:]:
        assert torch.equal(acc[0], b)


def test_sum_without_average():
    xs = _inputs(4, 1000, torch.float32)
    for algo in FLAT + HIER:
        bufs = [x.clone() for x in xs]
        virtual_allreduce(bufs, algo, average=False, local_size=2 if algo in HIER else None)
        assert torch.allclose(bufs[0].double(), torch.stack([x.double() for x in xs]).sum(0), atol=1e-4)


def _sends(text, step):
    line = [l for l in text.splitlines() if l.startswith(f"step {step}:")][0]
    return [(int(o), int(c)) for o, c in re.findall(r"send ->\d+ D@(\d+) x(\d+)", line)]


@pytest.mark.parametrize("N", [2, 3, 8])
def test_ring_geometry_matches_python_oracle(N):
    """C++ slicing == parallel/allreduce.py split_ranges, including numel < 64 * N (no rounding)."""
    for n in [1, 5, 63, 64 * N - 1, 64 * N + 1, 1000, 9000]:
        text = plan_text("ring", 0, N, n, channels=1)
        chunks = split_ranges(n, N)
        # ring position of rank 0 in the identity single-channel order is 0: step 0 sends chunk 0
        if N > 1 and chunks[0][1]:
            assert _sends(text, 0) == [chunks[0]], (n, text)
        # step i of the reduce-scatter sends chunk (-i) mod N
        for i in range(N - 1):
            o, l = chunks[(-i) % N]
            if l:
                assert (o, l) in _sends(text, i)


def test_schedule_errors_are_exceptions():
    C = _ext.require()
    with pytest.raises(RuntimeError):
        C.virtual_allreduce([torch.zeros(10), torch.zeros(11)], C.ALGO_RING)
    with pytest.raises(ValueError):  # world not a multiple of local_size
        virtual_allreduce([torch.zeros(10) for _ in range(6)], "hier_ring", local_size=4)


@pytest.mark.parametrize("N", [2, 3, 8])
def test_ring_pipe_structure_and_bitwise_equal_to_ring(N):
    """The pipelined ring: reduce-scatter sub-steps flagged to overlap the previous sub-step's
    reduce (the executor checks they touch disjoint memory and runs the deferred order), the first
    all-gather step joins them all, and the result equals the plain ring bit for bit (same chunks,
    same summation order)."""
    n = 100_003
    text = plan_text("ring_pipe", 1, N, n, channels=3)
    steps = [l for l in text.splitlines() if l.startswith("step ")]
    rs = 2 * (N - 1)
    assert len(steps) == rs + (N - 1)
    assert "overlaps" not in steps[0] and all("overlaps" in l for l in steps[1:rs])
    assert not any("overlaps" in l for l in steps[rs:])
    for dtype in (torch.float32, torch.bfloat16):
        xs = _inputs(N, n, dtype, seed=3)
        a = [x.clone() for x in xs]
        b = [x.clone() for x in xs]
        virtual_allreduce(a, "ring", channels=3, accum_fp32=False)
        virtual_allreduce(b, "ring_pipe", channels=3, accum_fp32=False)
        for u, v in zip(a, b):
            assert torch.equal(u, v)
