"""Per-shape bandwidth of the 1x1-convolution GEMMs at the headline batch (ResNet-50, bs1280).

For every distinct 1x1 shape of the step (forward with BN statistics, data gradient with k-major
weights) times the production dispatch (``tile=0``: streaming kernel where served, else pick_tile) and
each tile configuration forced, streaming off and forced on. Prints one JSON line per shape with ms and
the TB/s of the compulsory bytes (A + B + C once), so the shapes far from the ~5.5 TB/s copy rate are
the targets. Interleaved in one process; medians of 15.

usage: python scripts/bench_gemm_bs1280.py [--batch 1280] [--out FILE.jsonl]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_learning_amd.ops import _ext  # noqa: E402

# name: (TileCfg, tile columns); a forced tile only runs where N is a whole number of its columns
TILES = {"128x128": (1, 128), "128x64": (2, 64), "256x128": (4, 128), "256x128w4": (5, 128), "128x256w4": (6, 256),
         "256x256": (8, 256)}


def timeit(fn, iters=15):
    for _ in range(3):
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


def shapes(batch):
    """(M, Cin, Cout, calls per step) of the ResNet-50 (v1.5) 1x1 convolutions."""
    m = {56: batch * 56 * 56, 28: batch * 28 * 28, 14: batch * 14 * 14, 7: batch * 7 * 7}
    out = {}

    def add(M, ci, co, n=1):
        out[(M, ci, co)] = out.get((M, ci, co), 0) + n

    cin = 64
    for hw, c, blocks in ((56, 64, 3), (28, 128, 4), (14, 256, 6), (7, 512, 3)):
        prev = hw * 2 if hw != 56 else 56
        add(m[prev], cin, c)                  # block 0 conv1 (stride on conv2)
        add(m[hw], cin, 4 * c)                # downsample (strided input subsampled first)
        add(m[hw], c, 4 * c, blocks)          # conv3
        add(m[hw], 4 * c, c, blocks - 1)      # conv1 of blocks 1..
        cin = 4 * c
    return sorted(out.items(), key=lambda kv: -kv[0][0] * (kv[0][1] + kv[0][2]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1280)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    C = _ext.require()
    dev = torch.device("cuda:0")
    rows = []
    for (M, Cin, Cout), calls in shapes(a.batch):
        for kind in ("fwd", "dgrad"):
            K, N = (Cin, Cout) if kind == "fwd" else (Cout, Cin)
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)
            # forward: W [N][K]; data gradient: k-major W [K][N]
            B = (torch.randn(N, K, device=dev) if kind == "fwd" else torch.randn(K, N, device=dev)).to(torch.bfloat16)
            kmaj = kind == "dgrad"
            stats = kind == "fwd"
            byts = (M * K + K * N + M * N) * 2
            r = {"kind": kind, "M": M, "K": K, "N": N, "calls": calls,
                 "stream_rows": C.gemm_stream_rows(M, N, K, K, N, kmaj), "pick_tile": C.pick_tile(M, N, K, True)}
            r["auto_ms"] = timeit(lambda: C.gemm_nt(A, B, stats, None, kmaj, 0))
            C.set_gemm_stream(0)
            r["nostream_ms"] = timeit(lambda: C.gemm_nt(A, B, stats, None, kmaj, 0))
            for name, (t, tbn) in TILES.items():
                if N % tbn:
                    continue
                try:
                    r[f"t{name}_ms"] = timeit(lambda: C.gemm_nt(A, B, stats, None, kmaj, t))
                except RuntimeError as e:  # shape not accepted by that tile
                    r[f"t{name}_ms"] = str(e)[:60]
            if K <= 256:
                C.set_gemm_stream(1)
                if C.gemm_stream_rows(M, N, K, K, N, kmaj):
                    r["stream_forced_ms"] = timeit(lambda: C.gemm_nt(A, B, stats, None, kmaj, 0))
            C.set_gemm_stream(-1)
            # the library GEMM (torch.matmul -> hipBLASLt) on the same operands, no BN-statistics epilogue
            Bt = B.t() if kind == "fwd" else B
            r["hipblaslt_ms"] = timeit(lambda: torch.matmul(A, Bt))
            r["auto_TBps"] = round(byts / r["auto_ms"] / 1e9, 2)
            r["auto_ms_per_step"] = round(r["auto_ms"] * calls, 4)
            rows.append(r)
            print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
            del A, B
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
