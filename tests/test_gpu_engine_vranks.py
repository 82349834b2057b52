"""The native engine's multi-rank schedules executed for N virtual ranks on ONE MI355X.

Every algorithm CommEngine runs at N > 1 (ring with 1..7 channels over edge-disjoint xGMI rings,
two-shot direct, central, RCCL-collective RS+AG, builtin, and the 2-step node reducer on P2P rings
or on sub-communicator collectives) runs here with its production Plan, chunk geometry and reduce
kernel (csrc/kernels/reduce.hip); links are device copies (csrc/comm/vexec.h). Checked against an
fp64 sum and bitwise against the host execution of the same plans; then whole GradSync steps of
N model replicas (TinyNet fp32, native-kernel ResNet-18 bf16 with fp32 accumulation).
Reference: /root/reference/src/allreduce.py:9-170, /root/reference/src/reducers.py:38-69.
"""
import copy

import pytest
import torch

from distributed_learning_amd.ops import _ext
from distributed_learning_amd.parallel.virtual import VirtualGroup, virtual_allreduce

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
ALGOS = ["builtin", "ring", "direct", "central", "rsag", "hier_ring", "hier_coll", "ring_pipe", "hier_central"]


def _inputs(N, n, dtype, seed=0):
    g = torch.Generator().manual_seed(seed * 7919 + n * 31 + N)
    return [(torch.randn(n, generator=g) * (1 + r)).to(dtype) for r in range(N)]


def _local(algo, N):
    if not algo.startswith("hier"):
        return None
    return 2 if N % 2 == 0 and N > 2 else N


@pytest.mark.parametrize("N", [2, 3, 4, 8])
@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_virtual_ranks_gpu_match_host_and_fp64(N, algo, dtype):
    _ext.require()
    sizes = [1, 7, 63, 64 * N - 1, 1000, 100_003] + (
        [4 * 1024 * 1024 + 37] if algo in ("ring", "hier_ring", "ring_pipe") else [])
    chans = range(1, 8) if algo in ("ring", "ring_pipe") and N == 8 else [0]
    for n in sizes:
        for ch in chans:
            if ch > 1 and n > 200_000 and ch not in (1, 7):
                continue
            xs = _inputs(N, n, dtype)
            gpu = [x.to(DEV) for x in xs]
            host = [x.clone() for x in xs]
            virtual_allreduce(gpu, algo, channels=ch, local_size=_local(algo, N))
            virtual_allreduce(host, algo, channels=ch, local_size=_local(algo, N))
            torch.cuda.synchronize()
            for r in range(N):
                g = gpu[r].cpu()
                if algo not in ("builtin", "rsag", "hier_coll"):  # collectives: emulation order, not RCCL's
                    assert torch.equal(g, host[r]), (algo, N, n, ch, r)
                assert torch.equal(g, gpu[0].cpu())
            ref = torch.stack([x.double() for x in xs]).mean(0)
            scale = torch.stack([x.double().abs() for x in xs]).mean(0) + 1e-30
            tol = (1e-5 if dtype == torch.float32 else 2.0 ** -8 * (N + 1)) * N
            assert float(((gpu[0].cpu().double() - ref).abs() / scale).max()) <= tol, (algo, N, n, ch)


def test_fp32_accumulation_of_bf16_buckets_gpu():
    N, n = 8, 1_000_003
    xs = _inputs(N, n, torch.bfloat16, seed=5)
    ref = torch.stack([x.double() for x in xs]).mean(0)
    for algo in ["ring", "direct", "hier_ring", "builtin"]:
        gpu = [x.to(DEV) for x in xs]
        host = [x.clone() for x in xs]
        virtual_allreduce(gpu, algo, local_size=4 if algo == "hier_ring" else None, accum_fp32=True)
        virtual_allreduce(host, algo, local_size=4 if algo == "hier_ring" else None, accum_fp32=True)
        g = gpu[3].cpu()
        if algo != "builtin":
            assert torch.equal(g, host[3]), algo
        half_ulp = ref.abs() * 2.0 ** -8
        assert bool(((g.double() - ref).abs() <= half_ulp * 1.001 + 1e-6).all()), algo


class _Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = torch.nn.Conv2d(3, 8, 3, padding=1)
        self.fc = torch.nn.Linear(8 * 8 * 8, 10)

    def forward(self, x):
        return self.fc(torch.relu(self.conv(x)).flatten(1))


@pytest.mark.parametrize("algo,local_size", [("ring", None), ("direct", None), ("hier_ring", 4), ("hier_coll", 2)])
def test_gradsync_virtual_ranks_gpu(algo, local_size):
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.parallel.grad_sync import GradSync

    N = 8
    torch.manual_seed(0)
    base = _Tiny().to(DEV)
    models = [copy.deepcopy(base) for _ in range(N)]
    group = VirtualGroup(N, algo, local_size=local_size, snapshot=True)
    syncs = [GradSync(m.parameters(), bucket_cap_bytes=4096, executor=group.executor(r)) for r, m in enumerate(models)]
    for r, (m, s) in enumerate(zip(models, syncs)):
        s.prepare()
        g = torch.Generator().manual_seed(r)
        x = torch.randn(4, 3, 8, 8, generator=g).to(DEV)
        y = torch.randint(0, 10, (4,), generator=g).to(DEV)
        cross_entropy(m(x), y).backward()
    for s in syncs:
        s.synchronize()
    torch.cuda.synchronize()
    assert len(group.inputs) == len(syncs[0].buckets) >= 2
    for k, ins in group.inputs.items():
        mean = torch.stack([t.double() for t in ins]).mean(0)
        for s in syncs:
            torch.testing.assert_close(s.buckets[k].flat.double(), mean, rtol=1e-5, atol=1e-7)
    for s in syncs:
        s.close()


def test_gradsync_virtual_ranks_native_resnet_bf16():
    """Native-kernel ResNet-18 (bf16 weights) replicas: every bucket ends as the fp32-accumulated
    average of the replicas' bf16 gradients, rounded once."""
    from distributed_learning_amd.models import resnet18
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.parallel.grad_sync import GradSync

    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        N = 4
        torch.manual_seed(0)
        base = resnet18().to(DEV).to(memory_format=torch.channels_last)
        dnn.bf16_weights(base)
        models = [copy.deepcopy(base) for _ in range(N)]
        group = VirtualGroup(N, "ring", accum_fp32=True, snapshot=True)
        syncs = [GradSync(m.parameters(), bucket_cap_bytes=4 << 20, executor=group.executor(r))
                 for r, m in enumerate(models)]
        for r, (m, s) in enumerate(zip(models, syncs)):
            s.prepare()
            g = torch.Generator().manual_seed(100 + r)
            x = torch.rand(8, 3, 64, 64, generator=g).to(DEV, torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            y = torch.randint(0, 1000, (8,), generator=g).to(DEV)
            cross_entropy(m(x), y).backward()
        for s in syncs:
            s.synchronize()
        torch.cuda.synchronize()
        assert len(group.inputs) == len(syncs[0].buckets)
        for k, ins in group.inputs.items():
            mean = torch.stack([t.double() for t in ins]).mean(0)
            out = syncs[0].buckets[k].flat.double()
            half_ulp = mean.abs() * 2.0 ** -8
            assert bool(((out - mean).abs() <= half_ulp * 1.001 + 1e-12).all()), k
            for s in syncs[1:]:
                assert torch.equal(s.buckets[k].flat, syncs[0].buckets[k].flat)
        for s in syncs:
            s.close()
    finally:
        dnn.set_backend("torch")
        dnn.set_native_conv(False)


def test_ring_step_launches_do_not_scale_with_channels():
    """One ring step = one launch for all links and one for all reduces, whatever the channel count
    (7 channels issued 7 reduce launches per step). The count comes from the engine's own
    issuing code (plan_exec.h LocalIssuer), which the virtual harness shares with CommEngine."""
    N, n = 8, 4 * 1024 * 1024
    bufs = [torch.randn(n, device=DEV) for _ in range(N)]
    counts = {ch: virtual_allreduce(bufs, "ring", channels=ch, average=False) for ch in (1, 3, 7)}
    assert counts[1] == counts[3] == counts[7] == 3 * (N - 1), counts
    # the pipelined ring: two sub-steps per reduce-scatter step, each one link + one reduce launch
    assert virtual_allreduce(bufs, "ring_pipe", channels=7, average=False) == 2 * 2 * (N - 1) + (N - 1)
