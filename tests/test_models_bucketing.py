"""Model definitions and the reference bucketizer."""
import pytest
import torch

from distributed_learning_amd.models import create_network, get_spec
from distributed_learning_amd.parallel.bucketing import ALIGN_ELEMS, bucketize, fusion_groups

MiB = 1024 * 1024


@pytest.mark.parametrize("name,tensors,params", [
    ("googlenet", 187, 13_004_888),
    ("googlenet_noaux", 173, 6_624_904),
    ("basicnet", 8, 1_199_882),
    ("resnet18", 62, 11_689_512),
    ("resnet18_cifar", 62, 11_181_642),
    ("resnet50", 161, 25_557_032),
    ("resnet152", 467, 60_192_808),
])
def test_param_counts(name, tensors, params):
    ps = list(create_network(name).parameters())
    assert len(ps) == tensors
    assert sum(p.numel() for p in ps) == params


def test_forward_shapes():
    for name, b in [("basicnet", 2), ("resnet18_cifar", 2), ("resnet18_cifar_stem", 2)]:
        spec = get_spec(name)
        m = create_network(name)
        out = m(torch.randn(b, *spec.input_shape))
        assert out.shape == (b, spec.num_classes)


def test_googlenet_aux_heads_unused():
    from distributed_learning_amd.parallel.grad_sync import find_unused_parameters

    m = create_network("googlenet")
    m.train()
    out = m(torch.randn(2, 3, 224, 224))
    assert out.shape == (2, 1000)
    unused = find_unused_parameters(out, list(m.parameters()))
    aux = {id(p) for n, p in m.named_parameters() if n.startswith("aux")}
    assert {id(p) for p in unused} == aux
    assert sum(p.numel() for p in unused) == 13_004_888 - 6_624_904


def _counts(name, sizes):
    ps = list(create_network(name).parameters())
    return [len(fusion_groups(ps, s)) for s in sizes]


def test_bucket_layout_googlenet_25mib():
    ps = list(create_network("googlenet").parameters())
    groups = fusion_groups(ps, 25 * MiB)
    assert [sum(p.numel() for p in g) for g in groups] == [5_242_040, 6_411_904, 1_350_944]
    assert len(fusion_groups(ps, 0)) == 187


@pytest.mark.parametrize("name,sizes,expected", [
    ("googlenet", [0, 64 * 1024, 256 * 1024, MiB, 4 * MiB, 16 * MiB, 25 * MiB, 64 * MiB],
     [187, 105, 67, 34, 13, 4, 3, 1]),
    ("googlenet_noaux", [0, 64 * 1024, 256 * 1024, MiB, 4 * MiB, 16 * MiB, 25 * MiB, 64 * MiB],
     [173, 93, 55, 25, 7, 2, 2, 1]),
    ("basicnet", [0, 64 * 1024, 256 * 1024, MiB, 4 * MiB, 16 * MiB, 25 * MiB, 64 * MiB], [8, 5, 3, 3, 3, 1, 1, 1]),
    ("resnet18", [0, MiB, 4 * MiB, 25 * MiB, 64 * MiB], [62, 22, 12, 2, 1]),
    ("resnet50", [0, MiB, 4 * MiB, 25 * MiB, 64 * MiB], [161, 66, 32, 5, 2]),
    ("resnet152", [0, MiB, 4 * MiB, 25 * MiB, 64 * MiB], [467, 252, 78, 10, 4]),
])
def test_bucket_counts_match_survey(name, sizes, expected):
    assert _counts(name, sizes) == expected


def test_bucket_rules():
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in (10, 1000, 3, 5000, 7)]
    # every bucket has >= 1 param, reverse order, oversize tensor alone
    groups = fusion_groups(ps, 4 * 1100)
    flat = [p for g in groups for p in g]
    assert flat == list(reversed(ps))
    assert all(len(g) >= 1 for g in groups)
    assert any(len(g) == 1 and g[0].numel() == 5000 for g in groups)
    bs = bucketize(ps, 4 * 1100)
    for b in bs:
        assert all(o % ALIGN_ELEMS == 0 for o in b.offsets)
        assert b.padded_numel >= b.numel


def test_fusion_off_launch_groups_are_consecutive_and_capped():
    """grad_sync.launch_groups: per-tensor buckets (fusion off) grouped per dtype, greedily in index order under
    the byte / tensor / span caps; an oversize tensor is alone; groups come in the order of their last member;
    a pure function of the parameter list."""
    import torch

    from distributed_learning_amd.models import resnet50
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.parallel.bucketing import bucketize
    from distributed_learning_amd.parallel.grad_sync import (LAUNCH_GROUP_BYTES, LAUNCH_GROUP_MAX, LAUNCH_GROUP_SPAN,
                                                             launch_groups)

    m = resnet50()
    dnn.bf16_weights(m)
    bs = bucketize(m.parameters(), 0)
    assert len(bs) == 161 and all(len(b.params) == 1 for b in bs)
    gs = launch_groups(bs)
    assert sorted(b.index for g in gs for b in g) == list(range(161))
    assert [g[-1].index for g in gs] == sorted(g[-1].index for g in gs)
    for g in gs:
        idx = [b.index for b in g]
        assert idx == sorted(idx) and idx[-1] - idx[0] < LAUNCH_GROUP_SPAN
        assert len({b.params[0].dtype for b in g}) == 1 and len(g) <= LAUNCH_GROUP_MAX
        nb = sum(b.padded_numel * b.params[0].element_size() for b in g)
        assert nb <= LAUNCH_GROUP_BYTES or len(g) == 1
    assert len(gs) < 161 / 2
    assert [[b.index for b in g] for g in launch_groups(bucketize(m.parameters(), 0))] == \
        [[b.index for b in g] for g in gs]
    assert torch.bfloat16 in {g[0].params[0].dtype for g in gs} and torch.float32 in {g[0].params[0].dtype for g in gs}
