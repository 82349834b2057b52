#!/usr/bin/env python3
"""Multi-process check of the native engine's IPC transport: N real processes, one GPU each or all
on one GPU (``--same_device 1``, the way a one-GPU box runs it; RCCL refuses that).

Launched with torch.distributed.run (``python scripts/ipc_engine_check.py --ranks 2`` starts the
ranks itself). Every rank all-reduces a rank-dependent, exactly representable pattern with every
schedule on the IPC transport (csrc/comm/ipc.h: pulls out of the peers' windows between flag
barriers), at odd sizes, fp32 and bf16 (fp32-staged), averaging and summing, checks the result
against the exact value, checks that all ranks hold bitwise identical results, and rank 0 prints
one JSON line. Reference schedules: /root/reference/src/allreduce.py:9-170.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ALGOS = ["builtin", "ring", "ring:1", "ring_pipe", "direct", "central", "rsag", "hier_ring", "hier_coll",
         "hier_central"]
SIZES = [1, 63, 4097, 1 << 20, 3_000_017]


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(a) -> int:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("DLA_COMM_TIMEOUT_S", "60")
    if a.same_device:
        env["DLA_SAME_DEVICE"] = "1"
    return subprocess.run(cmd, env=env, timeout=a.timeout).returncode


def worker(a) -> None:
    import torch
    import torch.distributed as dist

    from distributed_learning_amd.parallel import context as ctxmod

    same = os.environ.get("DLA_SAME_DEVICE") == "1"
    c = ctxmod.init(backend="gloo" if same else "nccl", same_device=same, transport="ipc")
    world, rank = c.world_size, c.rank
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    results = []
    for algo in a.algos.split(","):
        ls = 2 if (algo.startswith("hier") and world % 2 == 0 and world > 2) else None
        eng = c.engine(local_size=ls if ls else local, transport="ipc")
        for dtype in (torch.float32, torch.bfloat16):
            eng.set_accum_fp32(dtype == torch.bfloat16)
            for n in SIZES:
                for average in (True, False):
                    i = torch.arange(n, device=c.device, dtype=torch.int64)
                    pat = ((i % 7) - 3)
                    buf = (pat * (rank + 1)).to(dtype)
                    eng.allreduce(buf, algo, average)
                    eng.synchronize()
                    want = pat.double() * (world * (world + 1) / 2.0)
                    if average:
                        want = want / world
                    err = float((buf.double() - want).abs().max())
                    tol = 1e-6 if dtype == torch.float32 else float(want.abs().max()) * 2 ** -8 + 1e-6
                    gathered = [None] * world
                    dist.all_gather_object(gathered, buf.float().sum().item() if n else 0.0)
                    # bitwise agreement: compare a checksum of the raw bytes too
                    raw = buf.view(torch.int16 if dtype == torch.bfloat16 else torch.int32).long().sum().item()
                    raws = [None] * world
                    dist.all_gather_object(raws, raw)
                    results.append({"algo": algo, "dtype": str(dtype).split(".")[-1], "n": n, "average": average,
                                    "max_err": err, "ok": err <= tol and len(set(raws)) == 1})
    torch.cuda.synchronize()
    if rank == 0:
        bad = [r for r in results if not r["ok"]]
        print(json.dumps({"world": world, "same_device": same, "checked": len(results), "failed": bad[:20],
                          "ok": not bad}), flush=True)
    ctxmod.shutdown()
    if [r for r in results if not r["ok"]]:
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--same_device", type=int, default=1)
    ap.add_argument("--algos", default=",".join(ALGOS))
    ap.add_argument("--timeout", type=float, default=600.0)
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ:
        sys.exit(launch(a))
    worker(a)


if __name__ == "__main__":
    main()
