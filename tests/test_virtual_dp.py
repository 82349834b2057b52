"""Whole data-parallel steps on N virtual ranks in one process (CPU; GPU twin in
tests/test_gpu_engine_vranks.py): N model replicas, each with its own GradSync, buckets handed to
a VirtualGroup that all-reduces bucket k across the replicas with the native engine's schedules
once every replica produced it. Checks the reference's DP contract (/root/reference/src/ourdist.py,
/root/reference/src/allreduce.py): every replica ends with the exact average of the per-replica
gradients, N x batch b trains like 1 x batch N*b, and replicas stay bit-identical."""
import copy

import pytest
import torch

from distributed_learning_amd.ops import _ext
from distributed_learning_amd.parallel.grad_sync import GradSync
from distributed_learning_amd.parallel.virtual import VirtualGroup
from test_wrappers_dist import TinyNet, _data

pytestmark = pytest.mark.skipif(not _ext.available(), reason="native extension not built")


def virtual_step(models, group, seed, bucket_bytes=2048, device="cpu"):
    from distributed_learning_amd.ops.loss import cross_entropy

    syncs = [GradSync(m.parameters(), bucket_cap_bytes=bucket_bytes, executor=group.executor(r))
             for r, m in enumerate(models)]
    for r, (m, s) in enumerate(zip(models, syncs)):
        s.prepare()
        x, y = _data(r, seed=seed)
        cross_entropy(m(x.to(device)), y.to(device)).backward()
    for s in syncs:
        s.synchronize()
    for s in syncs:
        s.close()


def reference_mean_grads(base, world, seed):
    from distributed_learning_amd.ops.loss import cross_entropy

    acc = {}
    for r in range(world):
        m = copy.deepcopy(base)
        x, y = _data(r, seed=seed)
        cross_entropy(m(x), y).backward()
        for n, p in m.named_parameters():
            acc[n] = acc.get(n, 0) + p.grad.double() / world
    return acc


@pytest.mark.parametrize("world,algo,local_size", [
    (2, "ring", None), (4, "ring", None), (8, "ring", None), (3, "direct", None), (4, "central", None),
    (4, "builtin", None), (8, "rsag", None), (8, "hier_ring", 4), (8, "hier_coll", 2),
])
def test_virtual_ranks_average_exactly(world, algo, local_size):
    torch.manual_seed(0)
    base = TinyNet()
    models = [copy.deepcopy(base) for _ in range(world)]
    group = VirtualGroup(world, algo, local_size=local_size)
    virtual_step(models, group, seed=0)
    assert group.collectives >= 2  # several buckets at 2 KiB
    ref = reference_mean_grads(base, world, 0)
    for m in models:
        for n, p in m.named_parameters():
            torch.testing.assert_close(p.grad.double(), ref[n], rtol=1e-5, atol=1e-7)
    for m in models[1:]:
        for (n, p), q in zip(m.named_parameters(), models[0].parameters()):
            assert torch.equal(p.grad, q.grad), n


def test_virtual_training_equals_big_batch():
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.optim import FusedSGD

    world, steps = 4, 3
    torch.manual_seed(0)
    base = TinyNet()
    big = copy.deepcopy(base)
    models = [copy.deepcopy(base) for _ in range(world)]
    opts = [FusedSGD(m.parameters(), lr=0.1, momentum=0.5) for m in models]
    group = VirtualGroup(world, "ring", channels=3)
    for s in range(steps):
        virtual_step(models, group, seed=s)
        for o in opts:
            o.step()
    bopt = FusedSGD(big.parameters(), lr=0.1, momentum=0.5)
    for s in range(steps):
        xs, ys = zip(*[_data(r, seed=s) for r in range(world)])
        bopt.zero_grad()
        cross_entropy(big(torch.cat(xs)), torch.cat(ys)).backward()
        bopt.step()
    for (n, p), q in zip(big.named_parameters(), models[0].parameters()):
        torch.testing.assert_close(q, p, rtol=1e-4, atol=1e-5)
    for m in models[1:]:
        for p, q in zip(m.parameters(), models[0].parameters()):
            assert torch.equal(p, q)
