"""Helpers to run a function on N local Gloo ranks (CPU) via torch.multiprocessing.spawn."""
import os
import socket
import tempfile
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    import datetime

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    try:
        res = fn(rank, world, *args)
        torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
    except Exception:
        with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


def run(fn, world, *args, allow_missing: bool = False):
    """Run ``fn(rank, world, *args)`` on ``world`` Gloo ranks; return the list of results
    (``None`` for ranks that exited with status 0 without returning, when ``allow_missing``)."""
    with tempfile.TemporaryDirectory() as d:
        try:
            mp.start_processes(_entry, args=(world, free_port(), fn, args, d), nprocs=world, join=True,
                               start_method="spawn")
        except Exception:
            errs = [open(os.path.join(d, f)).read() for f in sorted(os.listdir(d)) if f.startswith("err")]
            raise RuntimeError("worker failed:\n" + "\n".join(errs))
        out = []
        for r in range(world):
            f = os.path.join(d, f"r{r}.pt")
            if allow_missing and not os.path.exists(f):
                out.append(None)
                continue
            out.append(torch.load(f, weights_only=False))  # written by this helper's own workers
        return out
