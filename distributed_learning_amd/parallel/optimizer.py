"""Horovod-style optimizer wrapper and state broadcast.

BASELINE.json asks for "the same DistributedOptimizer-wrapping API"; the reference itself wraps
the *model* (SURVEY.md §0). Both exist here:

    opt = dla.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.5),
                                   named_parameters=model.named_parameters())
    dla.broadcast_parameters(model.state_dict(), root_rank=0)
    dla.broadcast_optimizer_state(opt, root_rank=0)
    ...
    loss.backward()   # buckets are all-reduced while backward runs (post-accumulate hooks)
    opt.step()        # waits for the last bucket (stream-side on GPU), then updates

``DistributedOptimizer`` does not need the forward output, so unused parameters are handled by
``GradSync.flush()`` at ``step()``/``synchronize()`` (zero-filled and launched in bucket order).
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional, Tuple

import torch
import torch.distributed as dist

from .grad_sync import GradSync, make_executor
from .reducers import make_reducer


class DistributedOptimizer(torch.optim.Optimizer):
    """Wraps any ``torch.optim.Optimizer``; gradients are averaged across workers before step."""

    def __init__(self, optimizer: torch.optim.Optimizer, named_parameters: Optional[Iterable[Tuple[str, torch.Tensor]]] = None,
                 *, bucket_cap_mb: float = 25.0, algorithm: str = "ring", native: Optional[bool] = None,
                 backward_passes_per_step: int = 1, comm_dtype: Optional[torch.dtype] = None,
                 grad_as_bucket_view: Optional[bool] = None, reducer=None):
        # NOTE: deliberately not calling Optimizer.__init__: we proxy the wrapped optimizer's state.
        self.optimizer = optimizer
        if named_parameters is not None:
            params = [p for _, p in named_parameters]
        else:
            params = [p for g in optimizer.param_groups for p in g["params"]]
        dev = params[0].device
        if reducer is None:
            if native is None:
                native = dev.type == "cuda" and dist.is_initialized() and dist.get_backend() == "nccl"
            reducer = make_reducer("immediate", algorithm, native=native)
        self.reducer = reducer
        # backward_passes_per_step (Horovod): gradients of that many backward passes accumulate
        # locally and each parameter's bucket slot becomes ready on its last pass
        self.sync = GradSync(params, bucket_cap_bytes=int(bucket_cap_mb * 1024 * 1024),
                             executor=make_executor(reducer, dev, True), overlap=True,
                             grad_as_bucket_view=grad_as_bucket_view, comm_dtype=comm_dtype,
                             passes_per_step=backward_passes_per_step)
        self.backward_passes_per_step = backward_passes_per_step
        self.sync.prepare()

    # Optimizer protocol ------------------------------------------------------------------------
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    @property
    def defaults(self):
        return self.optimizer.defaults

    def state_dict(self):
        return self.optimizer.state_dict()

    def load_state_dict(self, sd):
        return self.optimizer.load_state_dict(sd)

    def add_param_group(self, group):
        raise RuntimeError("DistributedOptimizer: parameter groups are fixed at construction")

    def synchronize(self) -> None:
        self.sync.synchronize()

    def step(self, closure=None):
        self.synchronize()
        out = self.optimizer.step(closure) if closure is not None else self.optimizer.step()
        self.sync.prepare()
        return out

    def zero_grad(self, set_to_none: bool = True):
        # gradients live in (or are packed from) persistent buffers; prepare() zeroes them
        self.sync.prepare()

    def skip_synchronize(self):
        return self.sync.no_sync()

    def __repr__(self):
        return f"DistributedOptimizer({self.optimizer!r}, buckets={len(self.sync.buckets)})"


def broadcast_parameters(params, root_rank: int = 0, group=None) -> None:
    """Broadcast a ``state_dict()`` or an iterable of (name, tensor) / tensors from ``root_rank``."""
    if not dist.is_initialized() or dist.get_world_size(group) <= 1:
        return
    if isinstance(params, dict):
        items = list(params.values())
    else:
        items = [p[1] if isinstance(p, tuple) else p for p in params]
    with torch.no_grad():
        for t in items:
            if isinstance(t, torch.Tensor):
                dist.broadcast(t.data if t.is_leaf else t, src=root_rank, group=group)


def broadcast_optimizer_state(optimizer, root_rank: int = 0, group=None) -> None:
    """Broadcast optimizer tensor state (e.g. momentum buffers) and scalar hyper-parameters."""
    if not dist.is_initialized() or dist.get_world_size(group) <= 1:
        return
    opt = getattr(optimizer, "optimizer", optimizer)
    sd = opt.state_dict()
    hyper = [{k: v for k, v in g.items() if k != "params"} for g in sd["param_groups"]]
    obj = [hyper]
    dist.broadcast_object_list(obj, src=root_rank, group=group)
    for g, h in zip(opt.param_groups, obj[0]):
        g.update(h)
    # tensor state: every rank must hold the same keys; create on non-roots if missing
    for group_ in opt.param_groups:
        for p in group_["params"]:
            st = opt.state.get(p, {})
            keys = [sorted(k for k, v in st.items() if isinstance(v, torch.Tensor))]
            dist.broadcast_object_list(keys, src=root_rank, group=group)
            for k in keys[0]:
                if k not in st:
                    st[k] = torch.zeros_like(p)
                    opt.state[p] = st
                dist.broadcast(st[k], src=root_rank, group=group)


def allreduce(tensor: torch.Tensor, average: bool = True, group=None) -> torch.Tensor:
    """Horovod-style functional all-reduce (returns a new tensor)."""
    out = tensor.clone()
    allreduce_(out, average, group)
    return out


def allreduce_(tensor: torch.Tensor, average: bool = True, group=None) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(tensor, group=group)
        if average:
            tensor.div_(dist.get_world_size(group))
    return tensor


def allgather(tensor: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate ``tensor`` from every rank along dim 0."""
    if not dist.is_initialized() or dist.get_world_size(group) <= 1:
        return tensor.clone()
    outs = [torch.empty_like(tensor) for _ in range(dist.get_world_size(group))]
    dist.all_gather(outs, tensor.contiguous(), group=group)
    return torch.cat(outs, 0)


def broadcast(tensor: torch.Tensor, root_rank: int = 0, group=None) -> torch.Tensor:
    out = tensor.clone()
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(out, src=root_rank, group=group)
    return out
