"""Python front-end of the native RCCL comm engine (csrc/comm/engine.cpp).

One :class:`NativeEngine` per process group. Bootstrap: rank 0 of the group draws an RCCL unique
id, it is broadcast through ``torch.distributed`` (``broadcast_object_list`` on the group), and
every rank builds its own ``ncclComm_t`` plus a high-priority HIP stream. Ring channel orders are
computed once (:func:`edge_disjoint_rings`) and handed to C++.

Algorithm names map to the C++ schedules:
``builtin`` ncclAllReduce, ``ring`` multi-channel P2P ring, ``direct`` two-shot P2P,
``central`` parameter server, ``rsag`` ncclReduceScatter+ncclAllGather.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops import _ext
from .allreduce import edge_disjoint_rings

ALGO_CODES: Dict[str, str] = {
    "builtin": "ALGO_BUILTIN",
    "ring": "ALGO_RING",
    "ring_gpu": "ALGO_RING",
    "direct": "ALGO_DIRECT",
    "central": "ALGO_CENTRAL",
    "rsag": "ALGO_RSAG",
}


def algo_code(name: str) -> int:
    C = _ext.require()
    try:
        return int(getattr(C, ALGO_CODES[name]))
    except KeyError:
        raise ValueError(f"unknown native all-reduce algorithm {name!r}; choose from {sorted(ALGO_CODES)}") from None


class NativeEngine:
    """Wraps ``_C.CommEngine`` for one process group."""

    def __init__(self, impl, group, device: torch.device, channels: int):
        self.impl = impl
        self.group = group
        self.device = device
        self.channels = channels

    @classmethod
    def create(cls, group=None, device: Optional[torch.device] = None, channels: int = 0) -> "NativeEngine":
        C = _ext.require()
        group = group if group is not None else dist.group.WORLD
        ranks = dist.get_process_group_ranks(group) if group is not dist.group.WORLD else list(
            range(dist.get_world_size()))
        n = len(ranks)
        me = ranks.index(dist.get_rank())
        device = device or torch.device("cuda", torch.cuda.current_device())
        # Default channel count: one ring per outgoing xGMI link of a fully connected node (n-1).
        channels = channels or max(1, n - 1)
        rings = edge_disjoint_rings(n, channels)
        obj: List[object] = [C.CommEngine.get_unique_id() if me == 0 else None]
        dist.broadcast_object_list(obj, src=ranks[0], group=group)
        impl = C.CommEngine(me, n, obj[0], device.index, rings)
        return cls(impl, group, device, len(rings))

    # -- collectives -------------------------------------------------------------------------
    def allreduce(self, flat: torch.Tensor, algo: str = "builtin", average: bool = True) -> None:
        self.impl.allreduce(flat, algo_code(algo), average)

    def bucket_allreduce(self, flat: torch.Tensor, algo: str, average: bool = True, table=None,
                         pack_scale: float = 1.0, unpack_scale: float = 1.0) -> None:
        self.impl.bucket_allreduce(flat, algo_code(algo), average, table, pack_scale, unpack_scale)

    def bucket_allreduce_list(self, flat: torch.Tensor, algo: str, grads, offsets, average: bool = True) -> None:
        """Gather autograd-owned ``grads`` into ``flat`` at ``offsets`` on the comm stream, then reduce."""
        self.impl.bucket_allreduce_list(flat, algo_code(algo), average, list(grads), list(offsets))

    def broadcast(self, t: torch.Tensor, root: int = 0) -> None:
        self.impl.broadcast(t, root)

    def allgather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        self.impl.allgather(out, inp)

    # -- stream plumbing ---------------------------------------------------------------------
    def wait_on_current(self) -> None:
        self.impl.wait_on_current()

    def synchronize(self) -> None:
        self.impl.synchronize()

    def set_timing(self, on: bool) -> None:
        self.impl.set_timing(on)

    def consume_comm_ms(self) -> float:
        return float(self.impl.consume_comm_ms())

    def close(self) -> None:
        if self.impl is not None:
            self.impl.synchronize()
            self.impl = None
