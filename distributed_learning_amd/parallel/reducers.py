"""Reducers: how one fused gradient buffer is averaged across workers.

Reference (/root/reference/src/reducers.py):
* ``ReduceImmediatelly`` (1-step): ``put(buf)`` runs the all-reduce in the caller's thread and
  queues the buffer; ``get()`` dequeues it (reducers.py:6-19).
* ``NodeAggregateReducer`` / ``NodeAgreggateReducerCPU`` (2-step): workers push buffers through
  ``mp.Queue`` to a per-node parent that sums them on the CPU, divides by ``ndevs``, runs the
  inter-node all-reduce and hands the result back (reducers.py:21-69).

MI355X design (one process per GPU, no host staging):
* :class:`ImmediateReducer` — same contract; ``reduce(flat)`` averages over the whole group with
  any algorithm of :mod:`.allreduce` (or the native engine, see :class:`NativeReducer`).
* :class:`HierarchicalReducer` — the 2-step reducer as a device-side hierarchy: ring
  reduce-scatter inside the node (xGMI), all-reduce of each owned shard across nodes among ranks
  with the same local index, ring all-gather inside the node. Only 1/L of the bucket crosses the
  node boundary per GPU (vs the full bucket through one parent process in the reference).
  With one physical node it runs on "virtual nodes" (``local_size`` < world) for testing.
* :class:`NativeReducer` — the C++ RCCL engine; used on the comm stream by the stream executor.
"""
from __future__ import annotations

import queue
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

from .allreduce import Ring, get_algorithm


class Reducer:
    """Averages a flat buffer in place across the reducer's group."""

    native = False

    def reduce(self, flat: torch.Tensor) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    # reference-compatible queue API (reducers.py:11-19)
    def put(self, buf: torch.Tensor) -> None:
        self.reduce(buf)
        self._q().put(buf)

    def get(self) -> torch.Tensor:
        return self._q().get()

    def cleanup(self) -> None:
        pass

    def _q(self):
        if not hasattr(self, "_queue"):
            self._queue = queue.Queue(maxsize=1024)
        return self._queue


class ImmediateReducer(Reducer):
    """1-step reducer: every worker is a member of one flat all-reduce."""

    def __init__(self, algorithm: str | Callable = "ring", group=None, channels: int = 1):
        self.group = group
        self.algorithm = algorithm if isinstance(algorithm, str) else getattr(algorithm, "__name__", "custom")
        self.fn = get_algorithm(algorithm, channels) if isinstance(algorithm, str) else algorithm

    def reduce(self, flat: torch.Tensor) -> None:
        self.fn(flat, self.group)


# Reference spelling (reducers.py:6).
ReduceImmediatelly = ImmediateReducer


class HierarchicalReducer(Reducer):
    """2-step (node) reducer: intra-node RS -> inter-node all-reduce of shards -> intra-node AG."""

    def __init__(self, local_size: Optional[int] = None, inter_algorithm: str = "ring", channels: int = 1):
        world = dist.get_world_size()
        me = dist.get_rank()
        if local_size is None:
            import os

            local_size = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if world % local_size != 0:
            raise ValueError(f"world size {world} is not a multiple of local_size {local_size}")
        self.local_size = local_size
        self.num_nodes = world // local_size
        self.algorithm = inter_algorithm
        node, lr = divmod(me, local_size)
        # new_group must be called by every rank in the same order
        self.local_group = None
        for n in range(self.num_nodes):
            ranks = list(range(n * local_size, (n + 1) * local_size))
            g = dist.new_group(ranks)
            if n == node:
                self.local_group, self.local_ranks = g, ranks
        self.cross_group = None
        for l in range(local_size):
            ranks = [n * local_size + l for n in range(self.num_nodes)]
            g = dist.new_group(ranks)
            if l == lr:
                self.cross_group, self.cross_ranks = g, ranks
        self.local_ring = Ring(self.local_ranks, self.local_group, channels)
        self.inter = get_algorithm(inter_algorithm, channels)

    def reduce(self, flat: torch.Tensor) -> None:
        n = flat.numel()
        if self.local_size > 1:
            self.local_ring.reduce_scatter_(flat, scale_last=1.0 / self.local_size)
        if self.num_nodes > 1:
            slices = self.local_ring.owned_slices(n) if self.local_size > 1 else [(0, n)]
            for off, ln in slices:
                if ln:
                    self.inter(flat[off:off + ln], self.cross_group)
        if self.local_size > 1:
            self.local_ring.all_gather_(flat)


class NativeReducer(Reducer):
    """All-reduce through the C++ RCCL engine (stream-ordered on the engine's comm stream)."""

    native = True

    def __init__(self, engine, algorithm: str = "builtin"):
        self.engine = engine
        self.algorithm = algorithm

    def reduce(self, flat: torch.Tensor) -> None:
        self.engine.allreduce(flat, self.algorithm, True)
        self.engine.wait_on_current()


def make_reducer(kind: str = "immediate", algorithm: str = "ring", *, channels: Optional[int] = None,
                 native: bool = False, engine=None, local_size: Optional[int] = None, group=None) -> Reducer:
    """Factory used by the experiment runners and the public API.

    ``channels``: ring channels. ``None`` = the default (native engine: one ring per outgoing xGMI
    link, i.e. n - 1; Python rings: 1); an explicit count, including 1, is passed through."""
    if native:
        if engine is None:
            from .context import get_context

            engine = get_context().engine(local_size=local_size, channels=channels or 0)
        return NativeReducer(engine, algorithm)
    ch = 1 if channels is None else int(channels)
    if kind in ("immediate", "1step", "onestep"):
        return ImmediateReducer(algorithm, group, ch)
    if kind in ("hierarchical", "node", "2step", "twostep"):
        return HierarchicalReducer(local_size, algorithm, ch)
    raise ValueError(f"unknown reducer kind {kind!r}")
