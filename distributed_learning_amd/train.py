"""The per-worker training loop (reference: ``worker_process``, /root/reference/src/main.py:29-107).

Per batch, identical phase structure and timer names to the reference:
``batch`` ⊃ ``get_data`` -> ``data2dev`` -> ``zero_grad`` -> ``forward`` (model + loss) -> ``backprop``
-> ``sync`` (``model.sync_gradients()``) -> ``optimizer_step``, then one row appended with
``batch_count`` and ``data_len``; at the end ``{exp}_{node}_{worker}_times.csv``,
``{exp}_{node}_{worker}_loss.txt`` and ``{exp}_config.txt``.

Differences by design:
* errors propagate (the reference printed and swallowed them, main.py:109-114, which left the
  node pump blocked forever);
* the loss line is formatted from device values collected without a per-step host sync (the
  reference's f-string forced ``.item()`` every batch) unless ``--sync_timers 1``;
* a device-accurate ``*_device_times.csv`` (HIP events) is written beside the parity CSV;
* only one process writes ``{exp}_config.txt`` (the reference raced all workers on it);
* optional checkpoint save/resume (the reference had none);
* on GPU the step is the framework's measured headline path (the one ``bench.py`` times): native
  MFMA convolutions / FC heads and fused BN kernels, bf16 weights with fp32 master weights in the
  fused SGD (``--precision bf16``, default), on-device synthetic batches, and every gradient
  collective on the C++ RCCL engine's comm stream. ``--precision fp32`` runs the reference's
  numerics (fp32 weights and activations on MIOpen / torch kernels); ``--precision autocast`` keeps
  fp32 parameters under bf16 autocast.
"""
from __future__ import annotations

import datetime
import os
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from . import data as D
from .models import get_spec
from .ops import nn as dnn
from .ops.loss import cross_entropy
from .ops.optim import FusedSGD
from .timing import EventTimers, Timers
from .utils.log import Level, print_d


def _model_for(config, device):
    spec = get_spec(config.model_name)
    torch.manual_seed(config.seed)  # identical init on all ranks (reference main.py:31) ...
    model = spec.build().to(device)
    if _channels_last(config, device):
        model = model.to(memory_format=torch.channels_last)
    return spec, model


def _precision(config, device) -> str:
    return getattr(config, "precision", "fp32") if device.type == "cuda" else "fp32"


def _channels_last(config, device) -> bool:
    """NHWC on the GPU for the native (bf16) kernels; the fp32 reference-precision path keeps the
    reference's NCHW layout, where MIOpen has its tuned fp32 kernels (fp32 NHWC fell back to kernels
    that needed minutes per GoogLeNet step)."""
    return device.type == "cuda" and _precision(config, device) != "fp32"


def setup_compute_path(config, device) -> str:
    """Select the kernels of the step; returns the precision in effect (bf16 | autocast | fp32)."""
    prec = _precision(config, device)
    if device.type != "cuda":
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
        return prec
    # MIOpen's exhaustive find for the fp32 reference-precision path costs minutes of tuning per new
    # shape; its default (immediate-mode) choice is what the reference's own runs used
    torch.backends.cudnn.benchmark = prec != "fp32"
    native = config.kernels == "native" and prec != "fp32"  # the native kernels are bf16 kernels
    dnn.set_backend("native" if native else "torch")
    dnn.set_native_conv(native and getattr(config, "conv", "native") == "native")
    return prec


def _data_for(config, spec, device, rank: int, node_id: int, worker_id: int, dtype=torch.float32):
    if config.random_input or not config.dataset_root or not os.path.isdir(config.dataset_root):
        if not config.random_input:
            print_d(f"dataset root {config.dataset_root!r} not found: using synthetic data", Level.WARNING)
        return D.SyntheticBatches(config.batch_size, spec.input_shape, spec.num_classes, device,
                                  dtype=dtype, seed=config.seed, rank=rank,
                                  channels_last=_channels_last(config, device))
    ds = D.load_dataset(spec.dataset, config.dataset_root)
    return D.get_partition_loader(ds, node_id, worker_id, config.node_dev, config.total_dev, config.batch_size)


def save_checkpoint(path: str, model: nn.Module, optimizer, step: int, extra: Optional[dict] = None) -> None:
    """Rank-0 checkpoint: plain ``torch.save`` of state dicts (new functionality vs the reference)."""
    if dist.is_initialized() and dist.get_rank() != 0:
        return
    inner = getattr(model, "module", model)
    rng = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        rng["cuda"] = torch.cuda.get_rng_state()
    # the RNG state makes a resumed run draw the same dropout masks as an uninterrupted one
    state = {"model": inner.state_dict(), "optimizer": optimizer.state_dict(), "step": step, "extra": extra or {},
             "rng": rng}
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str, model: nn.Module, optimizer=None, map_location=None) -> int:
    """Load on every rank (``weights_only=True``: tensors and plain containers only)."""
    state = torch.load(path, map_location=map_location or "cpu", weights_only=True)
    inner = getattr(model, "module", model)
    inner.load_state_dict(state["model"])
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(state["optimizer"])
    rng = state.get("rng") or {}
    if "cpu" in rng:
        torch.set_rng_state(rng["cpu"].cpu())
    if "cuda" in rng and torch.cuda.is_available():
        torch.cuda.set_rng_state(rng["cuda"].cpu())
    return int(state.get("step", 0))


def worker_process(config, distribute_model: Callable, reducer, experiment_name: str,
                   node_id: Optional[int] = None, worker_id: Optional[int] = None) -> dict:
    rank = dist.get_rank() if dist.is_initialized() else 0
    node_id = rank // max(1, config.node_dev) if node_id is None else node_id
    worker_id = rank % max(1, config.node_dev) if worker_id is None else worker_id
    device = torch.device(f"cuda:{torch.cuda.current_device()}") if config.use_gpu else torch.device("cpu")
    print_d(f"Starting experiment {experiment_name} ({config.experiment}), {datetime.datetime.now()}", Level.INFO)
    prec = setup_compute_path(config, device)

    spec, model = _model_for(config, device)
    if prec == "bf16":
        dnn.bf16_weights(model)  # bf16 weights, fp32 masters in the optimizer (bench.py's path)
    model = distribute_model(model, reducer, config.grouping_size, device)
    params = list(getattr(model, "module", model).parameters())
    optimizer = FusedSGD(params, lr=config.lr, momentum=config.momentum, weight_decay=config.weight_decay,
                         master_weights=prec == "bf16")
    start_step = 0
    if getattr(config, "resume", None):
        start_step = load_checkpoint(config.resume, model, optimizer, map_location=device)
        print_d(f"resumed from {config.resume} at step {start_step}", Level.INFO)

    os.makedirs(config.folder, exist_ok=True)
    if rank == 0:
        with open(f"{config.folder}/{experiment_name}_config.txt", "w") as f:
            f.write(str(config))
    stem = f"{config.folder}/{experiment_name}_{node_id}_{worker_id}"
    sync_mode = int(config.sync_timers or 0)
    timers = Timers(sync=sync_mode == 1)
    batch_sync = sync_mode == 2 and device.type == "cuda"
    cl = _channels_last(config, device)
    ev = EventTimers() if device.type == "cuda" else None
    train_set = _data_for(config, spec, device, rank, node_id, worker_id,
                          dtype=torch.bfloat16 if prec == "bf16" else torch.float32)
    autocast = torch.autocast("cuda", dtype=torch.bfloat16) if prec == "autocast" \
        else torch.autocast("cpu", enabled=False)
    model.train()

    losses = []
    # a resumed run continues the original sequence: batch numbering, and the data stream position
    batch_count = start_step
    end_batch = start_step + config.limit_batches
    epoch0, skip = 0, 0
    sampler = getattr(train_set, "epoch_sampler", None)
    if isinstance(train_set, D.SyntheticBatches):
        train_set.seek(start_step)
    elif sampler is not None:
        # resume inside the same per-epoch order without loading the skipped batches
        epoch0, skip = D.resume_position(start_step, len(train_set))
    t_start = time.time()
    for epoch in range(epoch0, config.epoch_count):
        if batch_count >= end_batch:
            break
        if sampler is not None:
            sampler.set_epoch(epoch, skip * config.batch_size if epoch == epoch0 else 0)
        gen = iter(train_set)
        while batch_count < end_batch:
            timers.start("batch")
            ev and ev.start("batch")
            timers.start("get_data")
            nx = next(gen, None)
            if nx is None:
                break
            x, y = nx
            timers.end("get_data")

            timers.start("data2dev")
            x = x.to(device, non_blocking=True)
            y = y.to(device, non_blocking=True)
            if prec == "bf16" and x.is_floating_point() and x.dtype != torch.bfloat16:
                x = x.to(torch.bfloat16)
            if x.dim() == 4 and cl:
                x = x.contiguous(memory_format=torch.channels_last)
            timers.end("data2dev")

            timers.start("zero_grad")
            optimizer.zero_grad(set_to_none=True)
            timers.end("zero_grad")

            timers.start("forward")
            ev and ev.start("forward")
            with autocast:
                out = model(x)
                loss = cross_entropy(out, y)
            ev and ev.end("forward")
            timers.end("forward")

            timers.start("backprop")
            ev and ev.start("backprop")
            loss.backward()
            ev and ev.end("backprop")
            timers.end("backprop")

            timers.start("sync")
            ev and ev.start("sync")
            model.sync_gradients()
            ev and ev.end("sync")
            timers.end("sync")

            timers.start("optimizer_step")
            ev and ev.start("optimizer_step")
            optimizer.step()
            ev and ev.end("optimizer_step")
            timers.end("optimizer_step")

            losses.append(loss.detach().float())
            if sync_mode == 1:
                print_d(f"Worker {node_id}:{worker_id} loss for batch {batch_count}: {losses[-1].item()}", Level.DEBUG)
            elif batch_sync:
                torch.cuda.synchronize()  # the reference's per-batch loss print synchronised here (main.py:94-96)
            timers.end("batch")
            ev and ev.end("batch")
            extra = {"batch_count": batch_count, "data_len": x.size(0)}
            timers.end_experiment(experiment_name, extra)
            if ev:
                ev.end_experiment(experiment_name, extra)
            batch_count += 1

    if device.type == "cuda":
        torch.cuda.synchronize()
    wall = time.time() - t_start
    values = torch.stack(losses).cpu().tolist() if losses else []
    with open(f"{stem}_loss.txt", "w") as f:
        for i, v in enumerate(values):
            f.write(f"Worker {node_id}:{worker_id} loss for batch {start_step + i}: {v}\n")
    rows = timers.rows()
    timers.writeout(f"{stem}_times.csv")
    if ev:
        ev.writeout(f"{stem}_device_times.csv")
    if device.type == "cuda":
        from .ops import conv as nconv

        print_d(f"native conv dispatches ({experiment_name}): {dict(sorted(nconv.CALLS.items()))} "
                f"[precision {prec}, ops backend {dnn.get_backend()}, native conv {dnn.native_conv()}]", Level.INFO)
        nconv.CALLS.clear()
    if getattr(config, "checkpoint", None):
        save_checkpoint(config.checkpoint, model, optimizer, batch_count)
    model.cleanup()
    if hasattr(reducer, "cleanup"):
        reducer.cleanup()
    return {"losses": values, "rows": rows, "wall_s": wall, "batches": batch_count - start_step,
            "start_step": start_step}
