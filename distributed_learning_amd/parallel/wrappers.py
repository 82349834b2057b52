"""Data-parallel model wrappers with the reference's interface.

Reference (/root/reference/src/ourdist.py, /root/reference/src/main.py:181-196,239-248): a wrapper
is constructed as ``Wrapper(model, reducer, grouping_size, grad_buff_device)`` and exposes
``__call__/forward(data)``, ``sync_gradients()`` (called after ``loss.backward()``),
``cleanup()``, and attribute passthrough to the wrapped model. The strategies:

===================  =======================  ===============================================
reference            here                     strategy
===================  =======================  ===============================================
``OurDist``          :class:`PipelinedFusedDP` overlap (P) + fusion (F); grouping 0 = P only
``SeqMergeDist``     :class:`SequentialFusedDP` fusion only, reduce after backward
``SeqDist``          :class:`PerTensorDP`      one collective per tensor after backward
``WarmupDist``       :class:`WarmupDP`         forward once, then a cached zero output
DDP baseline         :class:`TorchDDP`         ``torch.nn.parallel.DistributedDataParallel``
``main_single``      :class:`SingleDevice`     no communication ("Ideal")
===================  =======================  ===============================================

All wrappers are ``nn.Module``s (the reference's GoogLeNet wrapper was not, which forced the DDP
``parameters`` monkey-patch at main.py:189) and broadcast rank 0's parameters and buffers at
construction (the reference relied on identical seeding only).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.bn_act import flush_bn_counters
from .executor import NullExecutor
from .grad_sync import GradSync, find_unused_parameters, make_executor
from .reducers import Reducer, make_reducer

DEFAULT_GROUPING = 25 * 1024 * 1024  # bytes (reference config.py:51)


def broadcast_module(module: nn.Module, root: int = 0, group=None) -> None:
    """Broadcast parameters and buffers from ``root`` (one flat collective per dtype/device)."""
    if not dist.is_initialized() or dist.get_world_size(group) <= 1:
        return
    tensors = [t for t in list(module.parameters()) + list(module.buffers())]
    by_key = {}
    for t in tensors:
        by_key.setdefault((t.dtype, t.device), []).append(t)
    host_staged = dist.get_backend(group) == "gloo"  # Gloo ranks sharing one GPU: move through the host
    for _, ts in by_key.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        if host_staged and flat.is_cuda:
            buf = flat.cpu()
            dist.broadcast(buf, src=root, group=group)
            flat.copy_(buf)
        else:
            dist.broadcast(flat, src=root, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


class _DPBase(nn.Module):
    def __init__(self, model: nn.Module, broadcast: bool = True):
        super().__init__()
        self.module = model
        if broadcast:
            broadcast_module(model)

    def forward(self, *args, **kw):
        return self.module(*args, **kw)

    def sync_gradients(self) -> None:
        pass

    def cleanup(self) -> None:
        pass

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.__dict__["_modules"]["module"], name)


def _resolve_reducer(reducer) -> Reducer:
    if reducer is None or isinstance(reducer, str):
        return make_reducer("immediate", reducer or "ring")
    return reducer


class PipelinedFusedDP(_DPBase):
    """Overlap + fusion (the reference's ``OurDist``)."""

    def __init__(self, model: nn.Module, reducer=None, grouping_size: int = DEFAULT_GROUPING,
                 grad_buff_device=None, *, find_unused_parameters: bool = False, static_graph: bool = False,
                 grad_as_bucket_view: Optional[bool] = None, comm_dtype: Optional[torch.dtype] = None,
                 overlap: bool = True, broadcast: bool = True):
        super().__init__(model, broadcast)
        self.reducer = _resolve_reducer(reducer)
        dev = next(model.parameters()).device
        if grad_buff_device is not None and torch.device(grad_buff_device) != dev:
            # The reference staged buckets in host memory (grad_buff_device="cpu", main.py:35);
            # on MI355X buckets live in HBM next to the gradients.
            pass
        self.find_unused = find_unused_parameters
        self.static_graph = static_graph
        self._unused_cache = None
        self.sync = GradSync(model.parameters(), bucket_cap_bytes=int(grouping_size),
                             executor=make_executor(self.reducer, dev, overlap), overlap=overlap,
                             grad_as_bucket_view=grad_as_bucket_view, comm_dtype=comm_dtype)

    @property
    def groups(self):
        return self.sync.buckets

    def forward(self, *args, **kw):
        self.sync.prepare()
        out = self.module(*args, **kw)
        flush_bn_counters()
        if self.find_unused and torch.is_grad_enabled():
            if self._unused_cache is None or not self.static_graph:
                self._unused_cache = find_unused_parameters(out, self.sync.params)
            self.sync.mark_ready(self._unused_cache)
        return out

    def sync_gradients(self) -> None:
        self.sync.synchronize()

    def no_sync(self):
        return self.sync.no_sync()

    def cleanup(self) -> None:
        self.sync.close()


class SequentialFusedDP(PipelinedFusedDP):
    """Fusion without overlap (the reference's ``SeqMergeDist``, ourdist.py:180-203)."""

    def __init__(self, model, reducer=None, grouping_size: int = DEFAULT_GROUPING, grad_buff_device=None, **kw):
        kw["overlap"] = False
        super().__init__(model, reducer, grouping_size, grad_buff_device, **kw)


class PerTensorDP(PipelinedFusedDP):
    """One collective per tensor after backward (the reference's ``SeqDist``, ourdist.py:205-225)."""

    def __init__(self, model, reducer=None, grouping_size: int = 0, grad_buff_device=None, **kw):
        kw["overlap"] = False
        super().__init__(model, reducer, 0, grad_buff_device, **kw)


class WarmupDP(_DPBase):
    """Runs the real forward once, then returns a cached zero output (ourdist.py:227-248)."""

    def __init__(self, model, reducer=None, grouping_size: int = 0, grad_buff_device=None, broadcast: bool = False):
        super().__init__(model, broadcast)
        self.out = None

    def forward(self, *args, **kw):
        if self.out is None:
            with torch.no_grad():
                o = self.module(*args, **kw)
            self.out = torch.zeros_like(o, requires_grad=True)
        return self.out


class SingleDevice(_DPBase):
    """No communication; the 'Ideal' single-device baseline (main.py:239-248).

    Gradients still live in one persistent flat buffer (zeroed by a single memset per step and
    stable across steps, so the fused optimizer's tensor table is built once)."""

    def __init__(self, model, reducer=None, grouping_size: int = 0, grad_buff_device=None):
        super().__init__(model, broadcast=False)
        self.sync = GradSync(model.parameters(), bucket_cap_bytes=1 << 62, executor=NullExecutor(),
                             overlap=False, grad_as_bucket_view=True)

    def forward(self, *args, **kw):
        self.sync.prepare()
        out = self.module(*args, **kw)
        flush_bn_counters()
        return out

    def sync_gradients(self) -> None:
        self.sync.flush()


class TorchDDP(_DPBase):
    """PyTorch DDP baseline (main.py:181-196): RCCL backend on GPU, Gloo on CPU."""

    def __init__(self, model, reducer=None, grouping_size: int = DEFAULT_GROUPING, grad_buff_device=None,
                 find_unused_parameters: bool = True, gradient_as_bucket_view: bool = True):
        super().__init__(model, broadcast=False)
        dev = next(model.parameters()).device
        # DDP's reducer hooks copy gradients into its buckets inside backward, on the compute stream,
        # without joining the late weight-gradient side stream (ops/conv.py WGRAD_DEFER): no deferral
        # while a DDP wrapper lives
        from ..ops import conv as _conv

        _conv.block_deferral()
        self._blocks_deferral = True
        self.ddp = nn.parallel.DistributedDataParallel(
            model, device_ids=[dev.index] if dev.type == "cuda" else None,
            bucket_cap_mb=max(grouping_size, 1) / 1024 / 1024, find_unused_parameters=find_unused_parameters,
            gradient_as_bucket_view=gradient_as_bucket_view)

    def forward(self, *args, **kw):
        return self.ddp(*args, **kw)

    def cleanup(self) -> None:
        if getattr(self, "_blocks_deferral", False):
            from ..ops import conv as _conv

            _conv.unblock_deferral()
            self._blocks_deferral = False


# Reference class names
OurDist = PipelinedFusedDP
SeqMergeDist = SequentialFusedDP
SeqDist = PerTensorDP
WarmupDist = WarmupDP
