"""Bucket-size cost model for the gradient all-reduce on an 8-GPU MI355X node (xGMI).

The reference picked its 25 MiB fusion size empirically on P100 + Gloo/IPoIB (config.py:51;
sweep in measurements/gpu1/results/fusion_experiment_ourdist_16_33723740). On
MI355X the trade-off has different constants, so the size is derived instead of copied:

* **Collective time** of one S-byte bucket, ``T(S) = alpha + beta * S``:

  - ``ring`` with C channels over edge-disjoint directed rings (csrc/comm/plan.cpp): 2(N-1) P2P
    steps, each one RCCL group launch plus one multi-lane local-op launch -> ``alpha = 2 (N-1) alpha_step``
    (alpha_step measured on the virtual-rank harness + an RCCL group input: ``measured_step_alpha_us``);
    every channel moves 2 (N-1)/N * S/C bytes through ONE xGMI link (≈153 GB/s each, 7 per GPU)
    -> ``beta = 2 (N-1) / N / (C * link_bw)``;
  - ``builtin`` (ncclAllReduce): RCCL drives all links itself; ``alpha`` = one launch,
    ``beta = 2 (N-1) / N / bus_bw`` with ``bus_bw`` the algorithm bandwidth RCCL reaches on the
    node (an input: measure it with the engine's comm-stream timers, ``allreduce_ms_per_step``).
  - fp32 accumulation of bf16 gradients (the engine default at N > 1) doubles S on the wire.

* **Overlap**: bucket k becomes ready at ``r_k`` during backward (when its last gradient is
  produced) and the comm stream runs buckets in order, so ``f_k = max(r_k, f_{k-1}) + T(S_k)``;
  the cost of a bucketing is the part of the last collective that sticks out past the end of
  backward, ``exposed = max(0, f_last - t_backward)`` — what the step actually pays.

Small buckets pay ``alpha`` many times; large ones start late (the first bucket waits for its
last gradient) and leave a long tail. Collectives running under backward are not free either: RCCL
kernels occupy CUs (one workgroup per channel) that the convolutions lose, so the objective adds
``contention * total collective time`` (default 0.06 ≈ 16 channel workgroups of 256 CUs). :func:`choose_bucket_cap` evaluates the reference's greedy
bucketizer (bucketing.py) at each candidate cap against gradient-ready times estimated from the
model's own per-layer FLOPs (:func:`ready_times_from_flops`, backward ≈ 2x forward FLOPs in
reverse layer order) and returns the cap with the least exposed time, preferring the smaller cap
within 1 %.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from .bucketing import fusion_groups

MiB = 1024 * 1024
XGMI_LINK_GBPS = 153.0  # one MI355X xGMI link, each direction
CANDIDATE_CAPS_MIB = (1, 2, 4, 8, 16, 25, 32, 64, 128, 256)


@dataclass(frozen=True)
class CollectiveModel:
    """T(S) = alpha_s + beta_s_per_byte * S."""
    name: str
    alpha_s: float
    beta_s_per_byte: float

    def time(self, nbytes: float) -> float:
        return self.alpha_s + self.beta_s_per_byte * nbytes


# Per-step issue cost of the engine's ring schedules, measured on the virtual-rank harness
# (scripts/vrank_ring_timing.py: the production execute_plan / LocalIssuer code with device copies as
# links, 8 ranks on one MI355X; fitted by scripts/fit_ring_alpha.py over 64 KiB .. 64 MiB buckets,
# profiles/r3/g12/vrank_eager.jsonl and profiles/r3/g08b/vrank_graph.jsonl): intercept / 2(N-1) steps.
# Eager = host issue + the step's multi-lane local-op launches; graph = device-side cost alone.
VRANK_STEP_ALPHA_US = {("ring", 1, "eager"): 5.3, ("ring", 7, "eager"): 16.1,
                       ("ring", 1, "graph"): 3.4, ("ring", 7, "graph"): 8.0}
# What the harness cannot see: one RCCL group (C sends + C receives) per step on a real node. An input,
# not a measurement (no multi-GPU node is available to the builder); replace it with a fitted value
# from the engine's comm-stream timers (allreduce_ms_per_step at two bucket sizes) when one is.
RCCL_GROUP_US = 8.0


def measured_step_alpha_us(channels: int, graph: bool = False) -> float:
    """Issue cost per ring step for C channels: linear between the measured 1- and 7-channel points,
    plus the RCCL group launch."""
    mode = "graph" if graph else "eager"
    a1, a7 = VRANK_STEP_ALPHA_US[("ring", 1, mode)], VRANK_STEP_ALPHA_US[("ring", 7, mode)]
    c = max(1, min(int(channels), 7))
    return a1 + (a7 - a1) * (c - 1) / 6.0 + RCCL_GROUP_US


def ring_model(world: int, channels: int = 7, link_gbps: float = XGMI_LINK_GBPS,
               step_alpha_us: Optional[float] = None, graph: bool = False) -> CollectiveModel:
    """Multi-channel P2P ring (the engine's ``ring``): 2(N-1) steps, S/C bytes per channel link.
    ``step_alpha_us`` defaults to :func:`measured_step_alpha_us` for the channel count."""
    n = max(1, world)
    if n == 1:
        return CollectiveModel("ring", 0.0, 0.0)
    c = max(1, min(channels, n - 1))
    if step_alpha_us is None:
        step_alpha_us = measured_step_alpha_us(c, graph)
    return CollectiveModel(f"ring{c}", 2 * (n - 1) * step_alpha_us * 1e-6,
                           2.0 * (n - 1) / n / (c * link_gbps * 1e9))


def builtin_model(world: int, bus_gbps: float = 300.0, alpha_us: float = 25.0) -> CollectiveModel:
    """ncclAllReduce with an (input) algorithm bandwidth ``bus_gbps`` on the node."""
    n = max(1, world)
    if n == 1:
        return CollectiveModel("builtin", 0.0, 0.0)
    return CollectiveModel("builtin", alpha_us * 1e-6, 2.0 * (n - 1) / n / (bus_gbps * 1e9))


def exposed_time(bucket_bytes: Sequence[float], ready_s: Sequence[float], backward_s: float,
                 model: CollectiveModel) -> Tuple[float, float]:
    """(exposed seconds after backward, total collective seconds) for buckets run in order."""
    finish = 0.0
    total = 0.0
    for nb, r in zip(bucket_bytes, ready_s):
        t = model.time(nb)
        total += t
        finish = max(finish, r) + t
    return max(0.0, finish - backward_s), total


def ready_times_from_flops(model: nn.Module, input_shape: Sequence[int], backward_s: float,
                           batch: int = 2) -> Dict[int, float]:
    """Estimated time (s, from the start of backward) at which each parameter's gradient is ready.

    Forward FLOPs of every Conv2d / Linear are recorded with hooks on a small CPU batch; backward
    visits the layers in reverse with ≈2x their forward FLOPs, so a layer's parameters are ready
    at the cumulative reverse-order FLOP fraction of ``backward_s``. Parameters of other modules
    (BatchNorm) inherit the time of the next conv/linear backward that follows them."""
    flops: List[Tuple[nn.Module, float]] = []

    def hook(mod, inp, out):
        if isinstance(mod, nn.Conv2d):
            k = mod.kernel_size[0] * mod.kernel_size[1] * mod.in_channels // mod.groups
            flops.append((mod, 2.0 * out.numel() * k))
        elif isinstance(mod, nn.Linear):
            flops.append((mod, 2.0 * out.numel() * mod.in_features))

    hs = [m.register_forward_hook(hook) for m in model.modules() if isinstance(m, (nn.Conv2d, nn.Linear))]
    dev = next(model.parameters()).device
    was = model.training
    try:
        model.train()
        with torch.no_grad():
            model(torch.zeros(batch, *input_shape, device=dev, dtype=next(model.parameters()).dtype))
    finally:
        model.train(was)
        for h in hs:
            h.remove()
    total = sum(f for _, f in flops) or 1.0
    t = 0.0
    ready: Dict[int, float] = {}
    for mod, f in reversed(flops):  # backward order
        t += f / total * backward_s
        for p in mod.parameters(recurse=False):
            ready.setdefault(id(p), t)
    # parameters of non-GEMM modules: ready with the earliest following GEMM backward in reverse
    # registration order (e.g. a BN's weight is produced just before its conv's backward)
    params = [p for p in model.parameters() if p.requires_grad]
    nxt = backward_s
    for p in params:  # forward order: a BN after conv l is ready when the backward reaches it,
        if id(p) in ready:  # i.e. before conv l finishes -> take conv l's time as an upper bound
            nxt = ready[id(p)]
        else:
            ready[id(p)] = nxt
    return ready


def evaluate_caps(params: Sequence[torch.Tensor], ready: Dict[int, float], backward_s: float,
                  model: CollectiveModel, caps_mib: Sequence[float] = CANDIDATE_CAPS_MIB,
                  wire_bytes_per_elem: Optional[int] = None) -> List[Dict[str, float]]:
    """Exposed / total collective time of the reference bucketizer at each cap."""
    out = []
    for cap in caps_mib:
        groups = fusion_groups(params, int(cap * MiB))
        nb = [sum(p.numel() * (wire_bytes_per_elem or p.element_size()) for p in g) for g in groups]
        rd = [max(ready.get(id(p), backward_s) for p in g) for g in groups]
        exp, tot = exposed_time(nb, rd, backward_s, model)
        out.append({"cap_mib": cap, "buckets": len(groups), "exposed_ms": exp * 1e3, "comm_ms": tot * 1e3})
    return out


def choose_bucket_cap(params: Sequence[torch.Tensor], ready: Dict[int, float], backward_s: float,
                      model: CollectiveModel, caps_mib: Sequence[float] = CANDIDATE_CAPS_MIB,
                      wire_bytes_per_elem: Optional[int] = None,
                      contention: float = 0.06) -> Tuple[float, List[Dict[str, float]]]:
    """The cap minimising exposed + contention x total collective time (smallest within 1 %)."""
    rows = evaluate_caps(params, ready, backward_s, model, caps_mib, wire_bytes_per_elem)
    for r in rows:
        r["cost_ms"] = r["exposed_ms"] + contention * r["comm_ms"]
    best = min(r["cost_ms"] for r in rows)
    for r in rows:
        if r["cost_ms"] <= best * 1.01 + 1e-9:
            return r["cap_mib"], rows
    return rows[-1]["cap_mib"], rows
