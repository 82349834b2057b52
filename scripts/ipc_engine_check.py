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


def _check(eng, c, dist, torch, algo, dtype, n, average, results, phase):
    world, rank = c.world_size, c.rank
    i = torch.arange(n, device=c.device, dtype=torch.int64)
    pat = ((i % 7) - 3)
    buf = (pat * (rank + 1)).to(dtype)
    eng.allreduce(buf, algo, average)
    eng.synchronize()
    want = pat.double() * (world * (world + 1) / 2.0)
    if average:
        want = want / world
    err = float((buf.double() - want).abs().max()) if n else 0.0
    tol = 1e-6 if dtype == torch.float32 else float(want.abs().max()) * 2 ** -8 + 1e-6
    # bitwise agreement across ranks: a checksum of the raw bytes
    raw = buf.view(torch.int16 if dtype == torch.bfloat16 else torch.int32).long().sum().item()
    raws = [None] * world
    dist.all_gather_object(raws, raw)
    results.append({"phase": phase, "algo": algo, "dtype": str(dtype).split(".")[-1], "n": n, "average": average,
                    "max_err": err, "ok": err <= tol and len(set(raws)) == 1})


def worker(a) -> None:
    import traceback

    import torch
    import torch.distributed as dist

    from distributed_learning_amd.parallel import context as ctxmod

    same = os.environ.get("DLA_SAME_DEVICE") == "1"
    c = ctxmod.init(backend="gloo" if same else "nccl", same_device=same, transport="ipc")
    world, rank = c.world_size, c.rank
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    results, engines, where = [], [], "setup"
    try:
        for algo in a.algos.split(","):
            ls = 2 if (algo.startswith("hier") and world % 2 == 0 and world > 2) else None
            eng = c.engine(local_size=ls if ls else local, transport="ipc")
            if eng not in engines:
                engines.append(eng)
            for dtype in (torch.float32, torch.bfloat16):
                eng.set_accum_fp32(dtype == torch.bfloat16)
                for n in SIZES:
                    for average in (True, False):
                        where = f"{algo} {dtype} n={n} average={average}"
                        _check(eng, c, dist, torch, algo, dtype, n, average, results, "sweep")
        # window lifecycle: every cycle replaces all windows by a new generation (a fresh nonce each,
        # read back through every peer's mapping) and runs two schedules through the new mappings
        eng = engines[0]
        for k in range(a.regrow):
            where = f"regrow cycle {k}"
            eng.remap_windows()
            for algo in ("direct", "ring"):
                _check(eng, c, dist, torch, algo, torch.float32, 4097 + 64 * k, True, results, f"regrow{k}")
    except Exception as e:  # noqa: BLE001 -- report which call failed on THIS rank, with the engine's record
        info = {}
        for eng in engines:
            try:
                info = eng.ipc_error_info()
            except Exception as e2:  # noqa: BLE001
                info = {"unavailable": str(e2)}
        print(json.dumps({"rank": rank, "failed_at": where, "error": f"{type(e).__name__}: {e}"[:2000],
                          "ipc": info}), file=sys.stderr, flush=True)
        traceback.print_exc()
        sys.exit(2)
    torch.cuda.synchronize()
    bad = [r for r in results if not r["ok"]]
    gens = engines[0].ipc_error_info() if engines else {}
    stale = sum(e.stale_mappings for e in engines)
    if bad:  # every rank names its own mismatches (rank 0's view alone hid the cause in r4 g23)
        print(json.dumps({"rank": rank, "failed": bad[:20], "ipc": gens}), file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps({"world": world, "same_device": same, "checked": len(results), "failed": bad[:20],
                          "regrow_cycles": a.regrow, "window_generation": gens.get("generation"),
                          "stale_mappings_refused": stale, "ok": not bad}), flush=True)
    ctxmod.shutdown()
    if bad:
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--same_device", type=int, default=1)
    ap.add_argument("--algos", default=",".join(ALGOS))
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--regrow", type=int, default=8, help="window generations to cycle through after the sweep")
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ:
        sys.exit(launch(a))
    worker(a)


if __name__ == "__main__":
    main()
