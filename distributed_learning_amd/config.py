"""Command-line configuration, compatible with the reference's positional CLI.

Reference (/root/reference/src/config.py:10-58): nine positionals ``size rank node_dev total_dev
master_addr ifname model_type dataset_root use_gpu`` (``size``/``rank`` may be ``envarg://VAR``)
and ``--job_id --experiment --limit_batches --backend --batch_size --random_input``; hard-coded
``epoch_count=100``, ``grouping_size=25 MiB``, ``lr=0.01``, ``momentum=0.5``, seed 1234.

Kept verbatim (same names, order, meaning), with the hard-coded values promoted to flags and the
MI355X options added (model override, dtype, all-reduce algorithm/channels, native engine,
kernel backend, timer mode). Positionals become optional when launched under ``torchrun`` (the
distributed environment supplies rank/size).
"""
from __future__ import annotations

import argparse
import os
from typing import List, Optional

from .utils.env import eval_arg

GROUPING_SIZE = 25 * 1024 * 1024
FUSION_TEST_SIZES_K = [256, 1024, 4 * 1024, 16 * 1024, 64 * 1024]  # reference main.py:287


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X distributed learning benchmark tool "
                                            "(reference-compatible CLI)")
    pos = [("size", "n", str, "number of nodes (or envarg://VAR)"),
           ("rank", "r", str, "rank (id) of this node (or envarg://VAR)"),
           ("node_dev", "d", int, "number of devices managed by this node"),
           ("total_dev", "D", int, "total number of devices"),
           ("master_addr", "a", str, "address of the master node"),
           ("ifname", "i", str, "network interface for Gloo (eg. lo, ib0, eth0)"),
           ("model_type", "M", str, "model: mnist | imagenet | resnet18 | resnet18_cifar | resnet50 | resnet152 ..."),
           ("dataset_root", "R", str, "root folder for the datasets"),
           ("use_gpu", "g", int, "whether to use the gpu (1) or just cpu (0)")]
    defaults = {"size": "envarg://WORLD_SIZE", "rank": "envarg://RANK", "node_dev": 1, "total_dev": None,
                "master_addr": "127.0.0.1", "ifname": "lo", "model_type": "mnist", "dataset_root": "../data",
                "use_gpu": None}
    for name, meta, typ, hlp in pos:
        p.add_argument(name, metavar=meta, type=typ, nargs="?", default=defaults[name], help=hlp)
    # reference optionals
    p.add_argument("--job_id", default="job", help="unique string used for the results folder name")
    p.add_argument("--experiment", default="main_ourdist", help="experiment function to run (see experiments.py)")
    p.add_argument("--limit_batches", type=int, default=3, help="number of batches to run")
    p.add_argument("--backend", default=None, help="torch.distributed backend (gloo | nccl); default by device")
    p.add_argument("--batch_size", type=int, default=128, help="per-worker batch size")
    p.add_argument("--random_input", type=int, default=0, help="1 = synthetic data (no dataset needed)")
    # promoted hard-coded values
    p.add_argument("--grouping_size", type=int, default=GROUPING_SIZE, help="fusion bucket size in bytes")
    p.add_argument("--epoch_count", type=int, default=100)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.5)
    p.add_argument("--weight_decay", type=float, default=0.0)
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--master_port", type=int, default=29501)
    # MI355X options
    p.add_argument("--model", default=None, help="model override (same names as model_type)")
    p.add_argument("--dtype", default=None, choices=["fp32", "bf16"],
                   help="compute dtype (bf16 on GPU by default, fp32 on CPU); fp32 = the reference's precision")
    p.add_argument("--precision", default=None, choices=["bf16", "autocast", "fp32"],
                   help="bf16: bf16 weights + fp32 master weights in the fused SGD, native kernels (GPU default; "
                        "the bench.py path); autocast: fp32 params under bf16 autocast; fp32: no reduced precision "
                        "(MIOpen / torch kernels, the reference's numerics)")
    p.add_argument("--conv", default="native", choices=["native", "miopen"],
                   help="convolutions / FC heads on the native MFMA kernels (bf16) or MIOpen")
    p.add_argument("--algorithm", default="ring", help="all-reduce algorithm: ring|builtin|central|direct|rsag")
    p.add_argument("--channels", type=int, default=0, help="ring channels (0 = one per xGMI peer)")
    p.add_argument("--native", type=int, default=None, help="1 = C++ RCCL engine (GPU default), 0 = torch.distributed")
    p.add_argument("--kernels", default=None, choices=["native", "torch"], help="model hot-path kernel backend")
    p.add_argument("--comm_dtype", default=None, choices=["fp32", "bf16"], help="gradient wire dtype")
    p.add_argument("--local_size", type=int, default=None, help="devices per (virtual) node for 2-step reducers")
    p.add_argument("--sync_timers", type=int, default=None,
                   help="0 = host timers only; 1 = synchronise the device at every timer; 2 = synchronise once at "
                        "the end of each batch, as the reference's per-batch loss print (.item()) did (GPU default)")
    p.add_argument("--hier_algorithm", default=None,
                   help="native engine algorithm of the 2-step runners (default hier_ring; hier_central for the "
                        "central runner; hier_coll = RCCL collectives on ncclCommSplit sub-communicators)")
    p.add_argument("--find_unused", type=int, default=None, help="graph walk for unused params each forward")
    p.add_argument("--results_root", default="results")
    p.add_argument("--checkpoint", default=None, help="path to save a checkpoint at the end of a run")
    p.add_argument("--resume", default=None, help="checkpoint to resume from")
    p.add_argument("--spawn", type=int, default=None,
                   help="1 = this process spawns node_dev local workers (reference launch style)")
    return p


def parse_args(argv: Optional[List[str]] = None):
    config = build_parser().parse_args(argv)
    return finalize(config)


def finalize(config):
    def _int_or(v, default):
        try:
            return int(eval_arg(v))
        except (KeyError, ValueError, TypeError):
            return default

    config.size = _int_or(config.size, 1)
    config.rank = _int_or(config.rank, 0)
    if config.total_dev is None:
        config.total_dev = config.size * config.node_dev
    if config.use_gpu is None:
        import torch

        config.use_gpu = 1 if torch.cuda.is_available() else 0
    model = config.model or config.model_type
    config.model_name = model
    config.epoch_count = int(config.epoch_count)
    if config.dtype is None:
        config.dtype = "fp32" if (not config.use_gpu or config.precision == "fp32") else "bf16"
    if config.precision is None:
        config.precision = "bf16" if config.dtype == "bf16" else "fp32"
    if not config.use_gpu:
        config.precision = "fp32"
    if config.sync_timers is None:
        config.sync_timers = 2 if config.use_gpu else 0
    if config.native is None:
        config.native = 1 if config.use_gpu else 0
    if config.kernels is None:
        config.kernels = "native" if config.use_gpu else "torch"
    if config.backend is None:
        config.backend = "nccl" if config.use_gpu else "gloo"
    if config.find_unused is None:
        config.find_unused = 1 if model in ("imagenet", "googlenet") else 0
    config.devices = [f"cuda:{i}" for i in range(config.node_dev)] if config.use_gpu else ["cpu"] * config.node_dev
    return config
