"""Single-GPU checks of the GPU data-parallel path (native RCCL engine at world size 1, gpu)."""
import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world1(cuda):
    from distributed_learning_amd.parallel import context as ctx

    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    c = ctx.init(backend="nccl")
    yield c
    ctx.shutdown()


def _train(model_fn, wrap, steps, bf16, shape=(3, 32, 32)):
    from distributed_learning_amd.data import SyntheticBatches
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    m = model_fn().to(dev).to(memory_format=torch.channels_last)
    if bf16:
        dnn.bf16_weights(m)
    w = wrap(m)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, master_weights=bf16)
    data = SyntheticBatches(8, shape, 10, dev, dtype=torch.bfloat16 if bf16 else torch.float32,
                            channels_last=True)
    losses = []
    for _ in range(steps):
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=not bf16):
            loss = cross_entropy(w(x), y)
        loss.backward()
        w.sync_gradients()
        opt.step()
        losses.append(float(loss))
    return m, losses


@pytest.mark.parametrize("arch,bf16,staged,grouping", [
    (a, b, s, g) for a in ("resnet18",) for b, s in [(False, False), (True, False), (True, True)]
    for g in (25 * 1024 * 1024, 64 * 1024, 0)] + [
    # GoogLeNet: fused Inception blocks, native stem, ceil-mode fused pools, and aux heads whose
    # parameters get no gradient (zero-filled by GradSync.flush before their bucket is reduced)
    ("googlenet", True, False, 1024 * 1024), ("googlenet", True, True, 1024 * 1024)])
def test_native_engine_steal_path_matches_single_device(world1, arch, bf16, staged, grouping):
    """Gather of autograd-owned grads into bucket buffers on the comm stream, the (world-1) RCCL
    all-reduce and the re-pointing of .grad at the averaged slots must give exactly the single-device
    update (the same kernels run; only the gradient storage differs)."""
    from distributed_learning_amd.models import googlenet, resnet18
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.parallel import PipelinedFusedDP, SingleDevice, make_reducer
    from distributed_learning_amd.parallel.executor import NativeStreamExecutor

    dnn.set_backend("native")
    native_conv = arch == "googlenet"
    dnn.set_native_conv(native_conv)
    # MIOpen picks non-deterministic conv algorithms by default (run-to-run differences of ~1e-3
    # that chaotic SGD amplifies); the comparison needs identical kernels on both sides.
    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        def wrap_dp(m):
            red = make_reducer("immediate", "builtin", native=True)
            w = PipelinedFusedDP(m, red, grouping, broadcast=False)
            # force the full multi-rank data path (pack -> collective -> re-point) on one GPU
            w.sync.executor = NativeStreamExecutor(red.engine, "builtin", passthrough=False)
            w.sync.passthrough = False
            if staged:  # the N>1 default: bf16 buckets gathered into fp32 staging, reduced, cast back
                red.engine.impl.set_force(True)
                red.engine.set_accum_fp32(True)
                w.sync.executor.reserve(w.sync.buckets)
            assert w.sync.grad_mode == "steal"
            return w

        build = (lambda: googlenet(10)) if arch == "googlenet" else (lambda: resnet18(10))
        shape = (3, 64, 64) if arch == "googlenet" else (3, 32, 32)
        m1, l1 = _train(build, wrap_dp, 4, bf16, shape)
        m2, l2 = _train(build, SingleDevice, 4, bf16, shape)
    finally:
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det
    assert l1 == pytest.approx(l2, rel=1e-5, abs=1e-5)
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.parametrize("staged", [False, True])
def test_fusion_off_launch_groups_match_single_device(world1, staged):
    """Fusion off (one bucket per tensor) on the native engine: consecutive per-tensor buckets are launched
    in groups (grad_sync.LaunchGroup -> engine.bucket_allreduce_group: one gather, one staging cast, one RCCL
    group of per-tensor all-reduces, one cast back). The forced world-1 path must reproduce the single-device
    update exactly, with fewer launches than tensors."""
    from distributed_learning_amd.models import resnet18
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.parallel import PipelinedFusedDP, SingleDevice, make_reducer
    from distributed_learning_amd.parallel.executor import NativeStreamExecutor

    dnn.set_backend("native")
    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    seen = {}
    try:
        def wrap_dp(m):
            red = make_reducer("immediate", "builtin", native=True)
            w = PipelinedFusedDP(m, red, 0, broadcast=False)
            if staged:
                red.engine.impl.set_force(True)
                red.engine.set_accum_fp32(True)
            w.sync.set_executor(NativeStreamExecutor(red.engine, "builtin", passthrough=False))
            seen["groups"], seen["buckets"] = len(w.sync.groups), len(w.sync.buckets)
            assert w.sync.grad_mode == "steal"
            return w

        m1, l1 = _train(lambda: resnet18(10), wrap_dp, 4, True)
        m2, l2 = _train(lambda: resnet18(10), SingleDevice, 4, True)
    finally:
        dnn.set_backend("torch")
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det
    assert 0 < seen["groups"] < seen["buckets"] == 62, seen
    assert l1 == pytest.approx(l2, rel=1e-5, abs=1e-5)
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=n)


def test_fusion_off_strict_one_collective_per_tensor(world1):
    """DLA_LAUNCH_GROUPS=0, the reference's fusion-off semantics (/root/reference/src/main.py:168-179,222-230;
    ourdist.py:54-68 with grouping_size=0): every gradient tensor is its own collective AND its own launch. On
    the forced world-1 data path (fp32 staging, RCCL 1-rank all-reduce) the engine's issue counters must show
    N launches of N collectives per step for N tensors in strict mode, fewer launches of the same N collectives
    in the grouped mode, and the two trainings must agree bit for bit."""
    from distributed_learning_amd import knobs
    from distributed_learning_amd.models import resnet18
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.parallel import PipelinedFusedDP, make_reducer
    from distributed_learning_amd.parallel.executor import NativeStreamExecutor

    dnn.set_backend("native")
    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    saved = knobs._CACHE.get("LAUNCH_GROUPS")
    out = {}
    try:
        for mode in ("1", "0"):
            knobs._CACHE["LAUNCH_GROUPS"] = mode
            seen = {}

            def wrap_dp(m, seen=seen):
                red = make_reducer("immediate", "builtin", native=True)
                w = PipelinedFusedDP(m, red, 0, broadcast=False)
                red.engine.impl.set_force(True)
                red.engine.set_accum_fp32(True)
                w.sync.set_executor(NativeStreamExecutor(red.engine, "builtin", passthrough=False))
                red.engine.impl.collective_counts(True)
                seen.update(groups=len(w.sync.groups), tensors=len(w.sync.buckets), engine=red.engine)
                return w

            m, losses = _train(lambda: resnet18(10), wrap_dp, 3, True)
            torch.cuda.synchronize()
            coll, units = (int(v) for v in seen["engine"].impl.collective_counts(True))
            out[mode] = dict(seen, coll=coll, units=units, losses=losses,
                             params=[p.detach().clone() for p in m.parameters()])
    finally:
        if saved is None:
            knobs._CACHE.pop("LAUNCH_GROUPS", None)
        else:
            knobs._CACHE["LAUNCH_GROUPS"] = saved
        dnn.set_backend("torch")
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det
    g, s = out["1"], out["0"]
    n = s["tensors"]
    assert n == g["tensors"] == 62
    assert s["groups"] == 0 and 0 < g["groups"] < n
    assert s["coll"] == 3 * n and s["units"] == 3 * n, s  # strict: one launch per tensor per step
    assert g["coll"] == 3 * n and g["units"] == 3 * g["groups"], g  # grouped: same collectives, fewer launches
    assert s["losses"] == g["losses"]
    for a, b in zip(s["params"], g["params"]):
        assert torch.equal(a, b)


def test_engine_algorithms_world1(world1):
    from distributed_learning_amd.parallel.engine import ALGO_CODES, NativeEngine

    eng = NativeEngine.create(dist.group.WORLD, torch.device("cuda:0"))
    x = torch.randn(100_003, device="cuda:0")
    for algo in sorted(set(ALGO_CODES)):
        y = x.clone()
        eng.allreduce(y, algo, True)
        eng.wait_on_current()
        torch.testing.assert_close(y, x)  # world size 1: average == identity
    eng.set_timing(True)
    eng.allreduce(x, "builtin", True)
    assert eng.consume_comm_ms() >= 0.0
    eng.close()
