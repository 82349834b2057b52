"""Co-run determinism: does a kernel give bitwise the same result when other kernels run concurrently on
another stream (as with the late-joined weight gradients) as when it runs alone? A difference means an
intra-kernel race whose outcome depends on timing (diagnosis helper, round 3 g23).

    python scripts/corun_determinism.py [--reps 15]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd.ops import _ext  # noqa: E402
from distributed_learning_amd.ops.conv import stem_pack_weight  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
CL = torch.channels_last


def rnd(*shape, scale=1.0):
    t = (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)
    return t.contiguous(memory_format=CL) if t.dim() == 4 else t


def flat(ts):
    return torch.cat([t.reshape(-1).float() for t in ts if t is not None])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    torch.manual_seed(0)
    x3 = rnd(16, 3, 224, 224)
    wpk = stem_pack_weight(rnd(64, 3, 7, 7, scale=0.1))
    xs = C.stem_fwd(x3, wpk, False)[2]
    dy112 = rnd(16, 64, 112, 112)
    x64, w64 = rnd(32, 64, 56, 56), rnd(64, 64, 3, 3, scale=0.05)
    x128, w128 = rnd(16, 128, 28, 28), rnd(128, 128, 3, 3, scale=0.05)
    x256 = rnd(32, 256, 14, 14)
    xs2, dys2 = rnd(16, 64, 56, 56), rnd(16, 128, 28, 28)
    A, B = rnd(100352, 256), rnd(256, 256, scale=0.05)
    victims = {
        "stem_fwd": lambda: flat(C.stem_fwd(x3, wpk, True)[:2]),
        "stem_wgrad": lambda: C.stem_wgrad(dy112, xs, 224, 224, torch.bfloat16),
        "conv3x3_fwd_64": lambda: flat(C.conv3x3_fwd(x64, w64, 1, True)),
        "conv3x3_fwd_128": lambda: flat(C.conv3x3_fwd(x128, w128, 1, True)),
        "conv3x3_dgrad_64": lambda: C.conv3x3_dgrad(x64, w64),
        "conv3x3_dgrad_128": lambda: C.conv3x3_dgrad(x128, w128),
        "conv3x3_wgrad_64 (halo)": lambda: C.conv3x3_wgrad(x64, x64, 1, torch.bfloat16),
        "conv3x3_wgrad_128": lambda: C.conv3x3_wgrad(x128, x128, 1, torch.bfloat16),
        "conv3x3_wgrad_256": lambda: C.conv3x3_wgrad(x256, x256, 1, torch.bfloat16),
        "conv3x3_wgrad_s2": lambda: C.conv3x3_wgrad(dys2, xs2, 2, torch.bfloat16),
        "gemm_nt_stats": lambda: flat(C.gemm_nt(A, B, True)),
        "gemm_tn": lambda: C.gemm_tn(A, A, torch.float32, 1.0),
    }
    big_a = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    big_b = torch.empty_like(big_a)

    def aggressor():  # weight gradients + a streaming copy, as on the side stream during backward
        C.conv3x3_wgrad(x64, x64, 1, torch.bfloat16)
        big_b.copy_(big_a)
        C.conv3x3_wgrad(x128, x128, 1, torch.bfloat16)

    other = torch.cuda.Stream(device=dev)
    bad = 0
    for name, fn in victims.items():
        ref = fn().clone()
        torch.cuda.synchronize()
        diffs, worst = 0, 0.0
        for r in range(a.reps):
            cur = torch.cuda.current_stream()
            other.wait_stream(cur)
            with torch.cuda.stream(other):
                for _ in range(2):
                    aggressor()
            out = fn()  # on the compute stream, overlapping the aggressor
            cur.wait_stream(other)
            torch.cuda.synchronize()
            if not torch.equal(out, ref):
                diffs += 1
                worst = max(worst, float((out.float() - ref.float()).abs().max()))
        bad += diffs
        print(f"{name:26s}: {diffs} / {a.reps} co-run repetitions differ from the solo run (max |diff| {worst:.3e})",
              flush=True)
    print("RESULT", "race" if bad else "clean", flush=True)


if __name__ == "__main__":
    main()
