"""Per-layer roofline benchmark of the native conv kernels at the headline config (ResNet-50, per-GPU
batch 512): every distinct conv shape, forward (with BN-statistics epilogue), data gradient and
weight gradient, timed with events (median of interleaved repeats, random operands).

Prints one JSON line per (layer, pass) with ms, achieved TB/s on the minimal byte count (read
operands once, write the result once) and TFLOP/s, then a table weighted by how often each shape
occurs in the network: where the step's conv time goes and how far each pass is from
max(bytes / 6 TB/s, flops / 2.5 PF).

    python scripts/bench_layers.py [--batch 512] [--out profiles/layers.jsonl] [--only fwd,dgrad,wgrad]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
HBM, PEAK = 6.0e12, 2.5e15


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def layers(B):
    """(name, kind, H_in, Cin, Cout, stride, count) of ResNet-50 v1.5 convs (torchvision layout)."""
    out = []
    cin = 64
    for H, w, n, s in [(56, 64, 3, 1), (28, 128, 4, 2), (14, 256, 6, 2), (7, 512, 3, 2)]:
        hin = H * s
        out.append((f"s{H}_c1_first", "1x1", hin, cin, w, 1, 1))
        out.append((f"s{H}_c2_first", "3x3", hin, w, w, s, 1))
        out.append((f"s{H}_c3", "1x1", H, w, 4 * w, 1, n))
        out.append((f"s{H}_ds", "1x1", H, cin, 4 * w, 1, 1))  # on the subsampled input
        if n > 1:
            out.append((f"s{H}_c1", "1x1", H, 4 * w, w, 1, n - 1))
            out.append((f"s{H}_c2", "3x3", H, w, w, 1, n - 1))
        cin = 4 * w
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--pipe", type=int, default=-1, help="force the MFMA main loop (see set_mfma_pipeline)")
    ap.add_argument("--tile", type=int, default=0, help="force the fwd/dgrad tile config (0 = auto; see TileCfg)")
    a = ap.parse_args()
    C.set_mfma_pipeline(a.pipe)
    B = a.batch
    passes = a.only.split(",")
    recs = []
    for name, kind, H, Cin, Cout, s, count in layers(B):
        OH = H // s
        M_in, M_out = B * H * H, B * OH * OH
        K = Cin * (9 if kind == "3x3" else 1)
        flops = 2.0 * M_out * K * Cout
        torch.manual_seed(0)
        if kind == "1x1":
            X = torch.randn(M_out, Cin, device=dev).to(torch.bfloat16)
            W = (torch.randn(Cout, Cin, device=dev) * 0.05).to(torch.bfloat16)
            dY = torch.randn(M_out, Cout, device=dev).to(torch.bfloat16)
            fns = {"fwd": lambda: C.gemm_nt(X, W, True, None, False, a.tile),
                   "dgrad": lambda: C.gemm_nt(dY, W, False, None, True, a.tile),
                   "wgrad": lambda: C.gemm_tn(dY, X, torch.bfloat16, 1.0)}
            byts = {"fwd": (M_out * Cin + M_out * Cout + Cin * Cout) * 2,
                    "dgrad": (M_out * Cout + M_out * Cin + Cin * Cout) * 2,
                    "wgrad": (M_out * Cout + M_out * Cin) * 2 + Cin * Cout * 2}
        else:
            x = torch.randn(B, Cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            w = (torch.randn(Cout, Cin, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            dy = torch.randn(B, Cout, OH, OH, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            fns = {"fwd": lambda: C.conv3x3_fwd(x, w, s, True, a.tile),
                   "dgrad": (lambda: C.conv3x3_dgrad(dy, w, None, a.tile)) if s == 1 else (lambda: C.conv3x3s2_dgrad(dy, w, H, H)),
                   "wgrad": lambda: C.conv3x3_wgrad(dy, x, s, torch.bfloat16)}
            byts = {"fwd": (M_in * Cin + M_out * Cout + 9 * Cin * Cout) * 2,
                    "dgrad": (M_out * Cout + M_in * Cin + 9 * Cin * Cout) * 2,
                    "wgrad": (M_out * Cout + M_in * Cin + 9 * Cin * Cout) * 2}
        for p in passes:
            ms = timeit(fns[p])
            roof = max(byts[p] / HBM, flops / PEAK) * 1e3
            r = {"layer": name, "kind": kind, "pass": p, "count": count, "M": M_out, "K": K, "N": Cout,
                 "ms": round(ms, 4), "TBps": round(byts[p] / ms / 1e9, 3), "TFps": round(flops / ms / 1e9, 1),
                 "roof_ms": round(roof, 4), "of_roof": round(roof / ms, 3)}
            recs.append(r)
            print(json.dumps(r), flush=True)
        del fns
        torch.cuda.empty_cache()
    tot = sum(r["ms"] * r["count"] for r in recs)
    troof = sum(r["roof_ms"] * r["count"] for r in recs)
    print(f"\nconv time per step (weighted by layer count): {tot:.2f} ms; roofline {troof:.2f} ms "
          f"({troof / tot:.0%} of roof)")
    by = {}
    for r in recs:
        k = (r["kind"], r["pass"])
        by.setdefault(k, [0.0, 0.0])
        by[k][0] += r["ms"] * r["count"]
        by[k][1] += r["roof_ms"] * r["count"]
    for k, (t, rf) in sorted(by.items()):
        print(f"  {k[0]:4s} {k[1]:6s} {t:7.2f} ms  roof {rf:6.2f} ms  ({rf / t:.0%})")
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
