"""Uninitialised-memory probe of single native ops at the ResNet-18 layer2.0 shapes (round 3 g27)."""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
CL = torch.channels_last


def rnd(*shape):
    t = torch.randn(*shape, device=dev).to(torch.bfloat16)
    return t.contiguous(memory_format=CL) if t.dim() == 4 else t


def fill(on):
    torch.use_deterministic_algorithms(on, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = on


torch.manual_seed(0)
for n, cin, cout, h in [(16, 64, 128, 56), (16, 128, 256, 28), (16, 256, 512, 14), (8, 64, 128, 56)]:
    dy, w = rnd(n, cout, h // 2, h // 2), rnd(cout, cin, 3, 3)
    fill(False)
    ref = C.conv3x3s2_dgrad(dy, w, h, h).float()
    fill(True)
    got = C.conv3x3s2_dgrad(dy, w, h, h).float()
    fill(False)
    ok = torch.isfinite(got).all().item() and torch.equal(ref, got)
    bad = (~torch.isfinite(got)).nonzero()
    print(f"s2 dgrad n={n} cin={cin} cout={cout} h={h}: {'ok' if ok else 'BAD'}; non-finite {bad.shape[0]}"
          f" first {bad[:4].tolist()}", flush=True)
# the 1x1 stride-2 shortcut conv backward and the dual BN backward through autograd
from distributed_learning_amd.ops import nn as dnn  # noqa: E402
from distributed_learning_amd.ops import conv as nconv  # noqa: E402

dnn.set_backend("native")
dnn.set_native_conv(True)
conv = nn.Conv2d(64, 128, 1, stride=2, bias=False).to(dev).to(torch.bfloat16).to(memory_format=CL)
x = rnd(16, 64, 56, 56)
for on in (False, True):
    fill(on)
    xi = x.clone().requires_grad_(True)
    y, _ = nconv.conv1x1(xi, conv, want_stats=False)
    y.backward(rnd(*y.shape))
    torch.cuda.synchronize()
    print(f"1x1 s2 bwd fill={on}: dx finite {torch.isfinite(xi.grad).all().item()}", flush=True)
fill(False)

# the 1x1 data-gradient GEMM itself at that shape, streaming kernel on / off, and neighbouring M
for mode in (1, 0):
    C.set_gemm_stream(mode)
    for M, K, N in [(12544, 128, 64), (12544, 64, 64), (12544, 128, 128), (25088, 128, 64), (802816, 128, 64),
                    (12544, 256, 64)]:
        A, B = rnd(M, K), rnd(K, N)
        fill(False)
        ref = C.gemm_nt(A, B, False, None, True)[0].float()
        fill(True)
        got = C.gemm_nt(A, B, False, None, True)[0].float()
        fill(False)
        badr = (~torch.isfinite(got)).any(1).nonzero().flatten()
        rows = C.gemm_stream_rows(M, N, K, K, N, True, False)
        print(f"gemm_nt dgrad stream={mode} M={M} K={K} N={N} (stream rows {rows}): "
              f"{'ok' if torch.equal(ref, got) else 'BAD'}; non-finite rows {badr.numel()} first {badr[:6].tolist()}",
              flush=True)
C.set_gemm_stream(-1)
