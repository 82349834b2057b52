"""Teacher-forced, segment-by-segment parity of the native training step with fp32 PyTorch
(the whole-model bound was vacuous for the early layers).

The native path runs the full model once exactly as in training (cross-segment fusions included);
each segment is then re-run in fp32 PyTorch on the native path's own input and output gradient
(distributed_learning_amd/utils/parity.py). Every segment's output, input gradient and parameter
gradients must be within a fixed 2e-2 relative L2 error — including the stem / first conv, the stem
max-pool and stage 1 — with no bound derived from an autocast run.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

BOUND = 2e-2


@pytest.mark.parametrize("arch,batch", [("resnet50", 32), ("googlenet", 32)])
def test_teacher_forced_segments(cuda, arch, batch):
    from distributed_learning_amd import models
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.utils.parity import teacher_forced, worst

    torch.manual_seed(1234)
    model = getattr(models, arch)().to(cuda).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(batch, 3, 224, 224, generator=g).to(cuda)
    y = torch.randint(0, 1000, (batch,), generator=g).to(cuda)
    rows = teacher_forced(model, x, y)
    for r in rows:
        print({k: (round(v, 5) if isinstance(v, float) else v) for k, v in r.items()})
    names = [r["segment"] for r in rows]
    assert names[0] in ("stem", "stem1") and names[-1] == "head"
    assert rows[0]["dw"] > 0  # the first conv's weight gradient is checked, not skipped
    w, where = worst(rows)
    assert w <= BOUND, f"{arch}: worst segment error {w:.3g} at {where}"
