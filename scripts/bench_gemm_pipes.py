#!/usr/bin/env python3
"""Main-loop pipeline sweep of the 1x1 GEMMs that the auto policy sends to the register-staged 128x128 tile
(K <= 512, stages 2-4 at the headline batch): every pipeline (0 register staging, 2 / 3 LDS-DMA stages,
4 / 5 v2 schedule, 6 / 7 buffer-DMA schedule) at the 128x128 and the 8-wave 256x128 tiles, forward with BN
statistics and data gradient with k-major weights. Medians of 15; one JSON line per shape.

usage: python scripts/bench_gemm_pipes.py [--batch 1280]
"""
import argparse
import json
import os
import sys

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(_HERE))
sys.path.insert(0, _HERE)
from distributed_learning_amd.ops import _ext  # noqa: E402

from bench_gemm_bs1280 import shapes, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1280)
    a = ap.parse_args()
    C = _ext.require()
    dev = torch.device("cuda:0")
    C.set_gemm_stream(0)
    for (M, Cin, Cout), calls in shapes(a.batch):
        if M > 1003520:
            continue
        for kind in ("fwd", "dgrad"):
            K, N = (Cin, Cout) if kind == "fwd" else (Cout, Cin)
            if K > 512:
                continue
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)
            B = (torch.randn(N, K, device=dev) if kind == "fwd" else torch.randn(K, N, device=dev)).to(torch.bfloat16)
            kmaj, stats = kind == "dgrad", kind == "fwd"
            r = {"kind": kind, "M": M, "K": K, "N": N, "calls": calls}
            C.set_mfma_pipeline(-1)
            r["auto_ms"] = timeit(lambda: C.gemm_nt(A, B, stats, None, kmaj, 0))
            for tile, tname in ((1, "128x128"), (4, "256x128")):
                for p in (0, 2, 3, 4, 6, 7):
                    C.set_mfma_pipeline(p)
                    try:
                        r[f"{tname}_p{p}"] = round(timeit(lambda: C.gemm_nt(A, B, stats, None, kmaj, tile)), 4)
                    except RuntimeError as e:
                        r[f"{tname}_p{p}"] = str(e)[:40]
            C.set_mfma_pipeline(-1)
            print(json.dumps(r), flush=True)
            del A, B
            torch.cuda.empty_cache()
    C.set_gemm_stream(-1)


if __name__ == "__main__":
    main()
