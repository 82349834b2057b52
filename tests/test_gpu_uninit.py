"""No native kernel may depend on memory it never wrote (gpu): a training step with every allocation
NaN-filled (torch.use_deterministic_algorithms + fill_uninitialized_memory, which also covers at::empty in
the extension) must give bitwise the gradients of a normal step. ResNet-18 exercises the BasicBlock paths
(3x3-only blocks, the stride-2 1x1 shortcut's plain data gradient), ResNet-50 the bottleneck fusions.
The round-3 bug this pins: the streaming GEMM's K = 128 data gradient left 1/3 of its rows unwritten
(scripts/uninit_probe.py located it, profiles/r3/scc_clobber_fix.md)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model", ["resnet18", "resnet50"])
def test_step_independent_of_uninitialised_memory(cuda, model):
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
    from uninit_probe import run

    from distributed_learning_amd.ops import nn as dnn

    try:
        ref = run(model, 2, 8, False)
        got = run(model, 2, 8, True)
    finally:
        torch.use_deterministic_algorithms(False)
        torch.utils.deterministic.fill_uninitialized_memory = True
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
    for s, (a, b) in enumerate(zip(ref, got)):
        nonfinite = [n for n, t in b.items() if not torch.isfinite(t).all()]
        assert not nonfinite, f"step {s}: non-finite gradients {nonfinite[:6]}"
        differ = [n for n in a if not torch.equal(a[n], b[n])]
        assert not differ, f"step {s}: gradients depend on uninitialised memory: {differ[:6]}"
