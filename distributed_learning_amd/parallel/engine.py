"""Python front-end of the native RCCL comm engine (csrc/comm/engine.cpp).

One :class:`NativeEngine` per process group. Bootstrap: rank 0 of the group draws an RCCL unique
id, it is broadcast through ``torch.distributed`` (``broadcast_object_list`` on the group), and
every rank builds its own ``ncclComm_t`` plus a high-priority HIP stream. Ring channel orders are
computed once (:func:`edge_disjoint_rings`) and handed to C++.

Algorithm names map to the C++ schedules:
``builtin`` ncclAllReduce, ``ring`` multi-channel P2P ring, ``direct`` two-shot P2P,
``central`` parameter server, ``rsag`` ncclReduceScatter+ncclAllGather, ``hier_ring`` the 2-step
node reducer on P2P rings (intra-node RS -> inter-node ring all-reduce of the owned shard ->
intra-node AG), ``hier_coll`` the same hierarchy on RCCL collectives over ``ncclCommSplit``
sub-communicators (reference /root/reference/src/reducers.py:38-69, main.py:129-137),
``ring_pipe`` the ring with its reduce-scatter in half-chunk sub-steps whose reduce kernels run on
a side stream, overlapped with the next sub-step's transfer, ``hier_central`` the 2-step reducer with
a parameter server between nodes (reference ``main_central_reduce``, main.py:198-206).

Every schedule is a cached Plan (csrc/comm/plan.h); :mod:`.virtual` runs the identical plans for
N virtual ranks inside one process (one GPU or the CPU), which is how the N>1 paths are tested
on a one-GPU box.
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
    "hier_ring": "ALGO_HIER_RING",
    "hier_coll": "ALGO_HIER_COLL",
    "ring_pipe": "ALGO_RING_PIPE",
    "hier_central": "ALGO_HIER_CENTRAL",
}


def algo_code(name: str) -> int:
    C = _ext.require()
    try:
        return int(getattr(C, ALGO_CODES[name]))
    except KeyError:
        raise ValueError(f"unknown native all-reduce algorithm {name!r}; choose from {sorted(ALGO_CODES)}") from None


def topology(world: int, channels: int = 0, local_size: Optional[int] = None) -> Dict[str, object]:
    """Ring orders for a group of ``world`` ranks (``local_size`` per node), as the engine takes them.

    Default channel count: one ring per outgoing xGMI link of a fully connected node (n - 1, i.e.
    7 edge-disjoint rings on an 8-GPU MI355X node)."""
    import os

    if local_size is None:
        local_size = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if local_size <= 0 or local_size > world or world % local_size:
            local_size = world
    elif local_size <= 0 or local_size > world or world % local_size:
        raise ValueError(f"local_size {local_size} does not divide the group size {world}")
    channels = channels or max(1, min(world, 8) - 1)
    nodes = world // local_size
    return {
        "rings": edge_disjoint_rings(world, channels),
        "local_size": local_size,
        "local_rings": edge_disjoint_rings(local_size, min(channels, max(1, local_size - 1))),
        "node_rings": edge_disjoint_rings(nodes, min(channels, max(1, nodes - 1))),
    }


class NativeEngine:
    """Wraps ``_C.CommEngine`` for one process group."""

    def __init__(self, impl, group, device: torch.device, channels: int):
        self.impl = impl
        self.group = group
        self.device = device
        self.channels = channels

    @classmethod
    def create(cls, group=None, device: Optional[torch.device] = None, channels: int = 0,
               local_size: Optional[int] = None, accum_fp32: Optional[bool] = None) -> "NativeEngine":
        """``local_size``: ranks per node for the 2-step algorithms (default ``LOCAL_WORLD_SIZE`` or
        the group size); ``accum_fp32``: reduce bf16 buckets in fp32 (default: on when n > 1)."""
        C = _ext.require()
        group = group if group is not None else dist.group.WORLD
        ranks = dist.get_process_group_ranks(group) if group is not dist.group.WORLD else list(
            range(dist.get_world_size()))
        n = len(ranks)
        me = ranks.index(dist.get_rank())
        device = device or torch.device("cuda", torch.cuda.current_device())
        topo = topology(n, channels, local_size)
        obj: List[object] = [C.CommEngine.get_unique_id() if me == 0 else None]
        dist.broadcast_object_list(obj, src=ranks[0], group=group)
        impl = C.CommEngine(me, n, obj[0], device.index, topo["rings"], topo["local_size"], topo["local_rings"],
                            topo["node_rings"])
        impl.set_accum_fp32(n > 1 if accum_fp32 is None else bool(accum_fp32))
        return cls(impl, group, device, len(topo["rings"]))

    # -- setup -------------------------------------------------------------------------------
    def reserve(self, algo: str, sizes, dtype: torch.dtype) -> None:
        """Pre-build the plans of these bucket sizes and size the scratch buffer once."""
        self.impl.reserve(algo_code(algo), [int(s) for s in sizes], 1 if dtype == torch.bfloat16 else 0)

    def set_accum_fp32(self, on: bool) -> None:
        self.impl.set_accum_fp32(bool(on))

    def describe_plan(self, algo: str, n: int) -> str:
        return self.impl.describe_plan(algo_code(algo), int(n))

    def async_error(self) -> str:
        return self.impl.async_error()

    def abort(self) -> None:
        self.impl.abort()

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
            try:
                if not self.impl.aborted():
                    self.impl.synchronize()
            finally:
                self.impl = None
