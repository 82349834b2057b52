"""Stem forward at batch 1024: halo-tiled vs implicit-GEMM kernel (interleaved, median of 15)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd.ops import _ext  # noqa: E402
from distributed_learning_amd.ops.conv import stem_pack_weight  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
x = torch.randn(1024, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
wpk = stem_pack_weight((torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16))


def med(fn, iters=15):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


r = {0: [], 1: []}
for _ in range(3):
    for m in (0, 1):
        C.set_stem_halo(m)
        r[m].append(med(lambda: C.stem_fwd(x, wpk, True)))
C.set_stem_halo(-1)
print(json.dumps({"batch": 1024, "implicit_ms": min(r[0]), "halo_ms": min(r[1]),
                  "note": "includes the space-to-depth fold (same in both)"}), flush=True)
