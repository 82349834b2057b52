"""CPU checks of the deferred block-final BN apply's bookkeeping (ops/bn_act.py PendingApply, deferral_scope;
models/resnet.py): which blocks may defer, that deferral is confined to ResNet.forward's scope, and that the scope
materialises what is left. The kernels themselves are GPU-tested (tests/test_gpu_gemm_apply.py)."""
import torch

from distributed_learning_amd import knobs
from distributed_learning_amd.models.resnet import Bottleneck, resnet18, resnet50, resnet152
from distributed_learning_amd.ops import bn_act


def test_every_bottleneck_but_the_last_feeds_a_next_one():
    for ctor, n in ((resnet50, 16), (resnet152, 50)):
        m = ctor()
        blocks = [b for layer in (m.layer1, m.layer2, m.layer3, m.layer4) for b in layer]
        assert len(blocks) == n and all(isinstance(b, Bottleneck) for b in blocks)
        assert [b.defer_output for b in blocks] == [True] * (n - 1) + [False]
    r18 = resnet18()
    assert not any(getattr(b, "defer_output", False) for layer in (r18.layer1, r18.layer4) for b in layer)


def test_deferral_only_inside_the_scope():
    assert not bn_act.deferral_active()
    with bn_act.deferral_scope():
        assert bn_act.deferral_active() == knobs.flag("DEFER_APPLY")
        with bn_act.deferral_scope():  # nested model calls keep their own list
            assert len(bn_act._SCOPE) == 2
        assert len(bn_act._SCOPE) == 1
    assert not bn_act.deferral_active() and not bn_act._SCOPE


class _FakePending(bn_act.PendingApply):
    written = []

    def materialise(self):
        if self.y is not None:
            _FakePending.written.append(self.y)
        self.clear()


def test_scope_exit_materialises_what_is_left_and_clears_references():
    y1, y2 = torch.empty(2), torch.empty(3)
    with bn_act.deferral_scope():
        p1 = _FakePending(None, None, None, None, y1, None)
        p2 = _FakePending(None, None, None, None, y2, None)
        bn_act._defer_record(y1, p1)
        bn_act._defer_record(y2, p2)
        assert bn_act.pending_of(y1) is p1
        p1.clear()  # consumed by its GEMM
        assert bn_act.pending_of(y1) is None
    assert _FakePending.written == [y2]  # only the unconsumed one
    assert bn_act.pending_of(y2) is None and p2.x is None and p2.y is None


def test_cpu_forward_unchanged_inside_the_scope():
    torch.manual_seed(0)
    m = resnet50(num_classes=10).eval()
    x = torch.randn(2, 3, 64, 64)
    ref = m(x)
    blocks = [b for layer in (m.layer1, m.layer2, m.layer3, m.layer4) for b in layer]
    for b in blocks:
        b.defer_output = False
    assert torch.equal(m(x), ref)  # the torch path never defers
