"""Benchmark entry point (reference: /root/reference/src/main.py:321-333).

Two launch styles, both one process per device:

1. torchrun (recommended)::

       torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m distributed_learning_amd.main \\
           --model resnet50 --random_input 1 --experiment experiment2 --limit_batches 30

2. the reference's positional style (``python -m distributed_learning_amd.main n r d D a i M R g
   --experiment X``): ``n``/``r`` are the node count/rank (``envarg://`` allowed); this process
   spawns ``d`` local workers with global ranks ``r*d + i`` out of ``D`` — the reference spawned
   ``d`` workers per node the same way for its 2-step runners (main.py:129-137).

Results go to ``results/{experiment}_{total_dev}_{job_id}/`` (main.py:324).
"""
from __future__ import annotations

import os
import sys
import traceback

import torch
import torch.multiprocessing as mp

from . import experiments
from .config import parse_args
from .parallel import context as ctx
from .utils.log import Level, print_d


def _run_worker(config) -> None:
    c = ctx.init(backend=config.backend, master_addr=config.master_addr,
                 master_port=None if "MASTER_PORT" in os.environ else config.master_port,
                 ifname=config.ifname if config.ifname not in (None, "lo") else None)
    config.rank_global = c.rank
    try:
        fn = experiments.EXPERIMENTS.get(config.experiment)
        if fn is None:
            raise SystemExit(f"unknown experiment {config.experiment!r}; "
                             f"choose from {sorted(experiments.EXPERIMENTS)}")
        fn(config)
    finally:
        ctx.shutdown()


def _spawned(i: int, config, base_rank: int) -> None:
    os.environ["RANK"] = str(base_rank + i)
    os.environ["LOCAL_RANK"] = str(i)
    os.environ["WORLD_SIZE"] = str(config.total_dev)
    os.environ["LOCAL_WORLD_SIZE"] = str(config.node_dev)
    os.environ["MASTER_ADDR"] = config.master_addr
    os.environ["MASTER_PORT"] = str(config.master_port)
    try:
        _run_worker(config)
    except BaseException:
        traceback.print_exc()
        sys.stdout.flush()
        raise


def main(argv=None) -> int:
    config = parse_args(argv)
    config.folder = os.path.join(config.results_root, f"{config.experiment}_{config.total_dev}_{config.job_id}")
    os.makedirs(config.folder, exist_ok=True)
    under_launcher = "WORLD_SIZE" in os.environ and "RANK" in os.environ
    spawn = config.spawn if config.spawn is not None else (not under_launcher and config.node_dev > 1)
    print_d(f"Number of available devices {torch.cuda.device_count() if config.use_gpu else 0}", Level.INFO)
    if spawn:
        base = config.rank * config.node_dev
        mp.start_processes(_spawned, args=(config, base), nprocs=config.node_dev, start_method="spawn", join=True)
    else:
        if not under_launcher:
            os.environ.setdefault("RANK", str(config.rank))
            os.environ.setdefault("WORLD_SIZE", str(config.total_dev))
        _run_worker(config)
    return 0


if __name__ == "__main__":
    sys.exit(main())
