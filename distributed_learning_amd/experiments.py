"""Experiment runners and suites with the reference's names (/root/reference/src/main.py:116-301).

Each ``main_*`` composes wrapper x reducer x all-reduce exactly as the reference's matrix
 and runs :func:`train.worker_process` in *this* process (one process per
device). Differences:
* the 2-step ("node reducer") runners are a device-side hierarchy — intra-node reduce-scatter
  over xGMI, inter-node all-reduce of the owned shards, intra-node all-gather — instead of a
  per-node parent process pumping CPU buffers through ``mp.Queue`` (reducers.py:38-69). On GPU they
  run on the C++ RCCL engine's native 2-step plans (``hier_ring`` for the ring runners,
  ``hier_central`` for ``main_central_reduce``, ``--hier_algorithm hier_coll`` for RCCL collectives
  on ncclCommSplit sub-communicators) with ``local_size`` = ``--local_size`` / ``node_dev`` /
  ``LOCAL_WORLD_SIZE``; on CPU (and with ``--native 0``) on :class:`HierarchicalReducer`;
* on GPU the 1-step runners go through the C++ RCCL engine (``--native 1``) so the collective
  runs on a dedicated HIP stream; ``--native 0`` uses the torch.distributed algorithms;
* ``main_seq`` sets ``experiment_name = "seq"`` (the reference forgot to, main.py:149-156).
New runners: ``main_onestep_builtin``/``_direct``/``_rsag`` (other engine algorithms),
``experiment_algorithms`` (all of them back to back), ``fusion_experiment_onestep``.
"""
from __future__ import annotations

import copy
import os

import torch.distributed as dist

from .config import FUSION_TEST_SIZES_K
from .parallel import (PerTensorDP, PipelinedFusedDP, SequentialFusedDP, SingleDevice, TorchDDP, WarmupDP,
                       make_reducer)
from .train import worker_process


class _NoReducer:
    def cleanup(self):
        pass


def _local_size(config) -> int:
    if config.local_size:
        return int(config.local_size)
    if config.node_dev and config.node_dev > 1:
        return int(config.node_dev)
    return int(os.environ.get("LOCAL_WORLD_SIZE", dist.get_world_size() if dist.is_initialized() else 1))


def _reducer(config, kind: str, algorithm: str):
    native = bool(config.native) and bool(config.use_gpu)
    ch = config.channels or (max(1, dist.get_world_size() - 1) if dist.is_initialized() else 1)
    if kind == "hierarchical":
        if native:
            algo = config.hier_algorithm or ("hier_central" if algorithm == "central" else "hier_ring")
            return make_reducer("hierarchical", algo, native=True, local_size=_local_size(config),
                                channels=config.channels)
        return make_reducer("hierarchical", algorithm, channels=1, local_size=_local_size(config))
    if native:  # the engine's default is one ring per outgoing link; an explicit --channels passes through
        return make_reducer("immediate", algorithm, channels=config.channels or None, native=True)
    return make_reducer("immediate", algorithm, channels=ch if algorithm.startswith("ring") else 1)


def _wrap(cls, config, **kw):
    comm_dtype = None
    if getattr(config, "comm_dtype", None) == "bf16":
        import torch

        comm_dtype = torch.bfloat16

    def distribute(model, reducer, grouping_size, device):
        extra = dict(kw)
        if cls in (PipelinedFusedDP, SequentialFusedDP, PerTensorDP):
            extra.setdefault("find_unused_parameters", bool(config.find_unused))
            extra.setdefault("static_graph", True)
            if comm_dtype is not None:
                extra["comm_dtype"] = comm_dtype
        return cls(model, reducer, grouping_size, device, **extra)

    return distribute


def _run(config, name, cls, reducer, grouping=None, **kw):
    cfg = copy.copy(config)
    if grouping is not None:
        cfg.grouping_size = grouping
    cfg.experiment_name = name
    return worker_process(cfg, _wrap(cls, cfg, **kw), reducer, name)


# ---- runners (reference main.py:116-248) ----------------------------------------------------------
def main_warmup(config):
    cfg = copy.copy(config)
    cfg.limit_batches = min(config.limit_batches, 3)
    return _run(cfg, "warmup", WarmupDP, _NoReducer())


def main_ourdist(config):
    return _run(config, "ourdist", PipelinedFusedDP, _reducer(config, "hierarchical", "ring"))


def main_ourdist_nccl(config):
    return _run(config, "ourdist_nccl", PipelinedFusedDP, _reducer(config, "hierarchical", "ring"))


def main_seq(config):
    return _run(config, "seq", PerTensorDP, _reducer(config, "hierarchical", "ring"))


def main_seq_merge(config):
    return _run(config, "seq_merge", SequentialFusedDP, _reducer(config, "hierarchical", "ring"))


def main_overlap(config):
    return _run(config, "overlap", PipelinedFusedDP, _reducer(config, "hierarchical", "ring"), grouping=0)


def main_ddp(config):
    return _run(config, "ddp", TorchDDP, _NoReducer())


def main_central_reduce(config):
    return _run(config, "central_node_reduce", PipelinedFusedDP, _reducer(config, "hierarchical", "central"))


def main_onestep_reduce(config):
    return _run(config, "onestep_reduce", PipelinedFusedDP, _reducer(config, "immediate", config.algorithm
                                                                          if config.algorithm else "ring"))


def main_onestep_central(config):
    return _run(config, "onestep_central", PipelinedFusedDP, _reducer(config, "immediate", "central"))


def main_onestep_overlap(config):
    return _run(config, "onestep_overlap", PipelinedFusedDP, _reducer(config, "immediate", "ring"), grouping=0)


def main_onestep_seq_merge(config):
    return _run(config, "onestep_seq_merge", SequentialFusedDP, _reducer(config, "immediate", "ring"))


def main_onestep_builtin(config):
    return _run(config, "onestep_builtin", PipelinedFusedDP, _reducer(config, "immediate", "builtin"))


def main_onestep_direct(config):
    return _run(config, "onestep_direct", PipelinedFusedDP, _reducer(config, "immediate", "direct"))


def main_onestep_rsag(config):
    if not (config.native and config.use_gpu):
        raise RuntimeError("rsag is a native-engine (GPU) algorithm")
    return _run(config, "onestep_rsag", PipelinedFusedDP, _reducer(config, "immediate", "rsag"))


def main_single(config):
    if dist.is_initialized() and dist.get_rank() != 0:
        return None  # the reference runs "single" on rank 0 only (main.py:248)
    return _run(config, "single", SingleDevice, _NoReducer())


# ---- suites (reference main.py:250-301) --------------------------------------------------------
def experiment1(config):
    main_warmup(config)
    main_ourdist(config)
    main_seq_merge(config)
    main_overlap(config)
    main_central_reduce(config)


def experiment2(config):
    main_warmup(config)
    main_ddp(config)
    main_onestep_reduce(config)
    main_onestep_central(config)


def experiment3(config):
    main_warmup(config)
    main_ddp(config)
    main_onestep_reduce(config)
    main_onestep_seq_merge(config)
    main_onestep_overlap(config)


def experiment_nccl(config):
    main_warmup(config)
    main_ddp(config)
    main_ourdist_nccl(config)


def experiment_ourdist_nccl(config):
    main_warmup(config)
    main_ourdist_nccl(config)


def experiment_single(config):
    main_warmup(config)
    main_single(config)


def experiment_onestep_central(config):
    main_warmup(config)
    main_onestep_central(config)


def experiment_algorithms(config):
    """Every 1-step algorithm back to back (new)."""
    main_warmup(config)
    main_onestep_builtin(config)
    main_onestep_reduce(config)
    main_onestep_direct(config)
    main_onestep_central(config)


def fusion_experiment(config, main_f):
    main_warmup(config)
    folder = config.folder
    for size_k in FUSION_TEST_SIZES_K:
        cfg = copy.copy(config)
        cfg.grouping_size = size_k * 1024
        cfg.folder = os.path.join(folder, f"{size_k}")
        os.makedirs(cfg.folder, exist_ok=True)
        main_f(cfg)


def fusion_experiment_ddp(config):
    fusion_experiment(config, main_ddp)


def fusion_experiment_ourdist(config):
    fusion_experiment(config, main_ourdist)


def fusion_experiment_onestep(config):
    fusion_experiment(config, main_onestep_reduce)


EXPERIMENTS = {k: v for k, v in globals().items() if (k.startswith("main_") or k.startswith("experiment")
                                                       or k.startswith("fusion_experiment")) and callable(v)}
