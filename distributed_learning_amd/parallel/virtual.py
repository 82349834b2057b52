"""Virtual ranks: the N>1 gradient path executed inside ONE process.

RCCL will not put two ranks on one GPU, and the GPU box has one MI355X, so the multi-rank
schedules of the C++ engine are exercised here: :func:`virtual_allreduce` runs the exact Plans
``CommEngine`` replays for N ranks (same chunk geometry, same edge-disjoint channel rings, same
reduce kernel, same fp32 staging of bf16 buckets) in lockstep, with device copies (GPU) or host
copies (CPU) as the links — see csrc/comm/vexec.h. A send without a matching receive, a length
mismatch or a receive overlapping a buffer the same step sends from raises instead of hanging.

:class:`VirtualGroup` lifts this to whole data-parallel steps: N model replicas in one process,
each with its own :class:`~.grad_sync.GradSync` whose executor hands complete buckets to the
group; bucket k is all-reduced across the N replicas' flat buffers as soon as every replica has
produced it, in bucket order — the same ordering contract RCCL imposes on real ranks.

Reference semantics being reproduced: /root/reference/src/allreduce.py:9-170 (ring, GPU ring,
central), /root/reference/src/reducers.py:38-69 (2-step node reducer).
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import torch

from ..ops import _ext
from .engine import algo_code, topology
from .executor import Executor


def virtual_allreduce(bufs: Sequence[torch.Tensor], algorithm: str = "ring", average: bool = True,
                      channels: int = 0, local_size: Optional[int] = None, accum_fp32: bool = False) -> int:
    """All-reduce ``bufs`` (one tensor per virtual rank) in place with the engine's schedules.

    GPU buffers run through the engine's own issuing code (csrc/comm/plan_exec.h); returns the
    number of kernel launches the links and local ops took (0 for host buffers)."""
    C = _ext.require()
    n = len(bufs)
    topo = topology(n, channels, local_size if local_size is not None else n)
    return C.virtual_allreduce(list(bufs), algo_code(algorithm), bool(average), topo["rings"], topo["local_size"],
                        topo["local_rings"], topo["node_rings"], bool(accum_fp32))


def ipc_host_allreduce(bufs: Sequence[torch.Tensor], algorithm: str = "ring", average: bool = True,
                       channels: int = 0, local_size: Optional[int] = None, accum_fp32: bool = False,
                       timeout_s: float = 30.0) -> None:
    """All-reduce host ``bufs`` with the IPC transport's protocol (csrc/comm/ipc.h): one thread per
    rank, each pulling from the peers' windows between flag barriers, exactly the schedule matching
    and barrier sequence the GPU transport issues -- checked here under real concurrency. A
    protocol bug surfaces as a wrong result or a barrier timeout, never a hang."""
    C = _ext.require()
    n = len(bufs)
    topo = topology(n, channels, local_size if local_size is not None else n)
    C.ipc_host_allreduce(list(bufs), algo_code(algorithm), bool(average), topo["rings"], topo["local_size"],
                         topo["local_rings"], topo["node_rings"], bool(accum_fp32), float(timeout_s))


def plan_text(algorithm: str, rank: int, world: int, n: int, channels: int = 0,
              local_size: Optional[int] = None, average: bool = True) -> str:
    """The schedule rank ``rank`` of ``world`` runs for an ``n``-element all-reduce (debugging)."""
    C = _ext.require()
    topo = topology(world, channels, local_size if local_size is not None else world)
    return C.plan_describe(algo_code(algorithm), rank, world, n, topo["rings"], topo["local_size"],
                           topo["local_rings"], topo["node_rings"], average)


class VirtualGroup:
    """N virtual data-parallel ranks sharing one process; hands out one executor per rank."""

    def __init__(self, world: int, algorithm: str = "ring", channels: int = 0, local_size: Optional[int] = None,
                 accum_fp32: bool = False, snapshot: bool = False):
        self.world = world
        self.snapshot = snapshot
        self.inputs: Dict[int, list] = {}  # bucket index -> per-rank flat copies before the reduce
        self.algorithm = algorithm
        self.channels = channels
        self.local_size = local_size
        self.accum_fp32 = accum_fp32
        self._pending: Dict[int, Dict[int, object]] = {}
        self._done: Dict[int, int] = {}
        self.collectives = 0

    def executor(self, rank: int) -> "VirtualExecutor":
        return VirtualExecutor(self, rank)

    def _submit(self, rank: int, b) -> None:
        slot = self._pending.setdefault(b.index, {})
        if rank in slot:
            raise RuntimeError(f"virtual rank {rank} submitted bucket {b.index} twice")
        slot[rank] = b
        if len(slot) == self.world:
            from .executor import BucketIO

            if self.snapshot:
                self.inputs[b.index] = [slot[r].flat.clone() for r in range(self.world)]
            virtual_allreduce([slot[r].flat for r in range(self.world)], self.algorithm, True, self.channels,
                              self.local_size, self.accum_fp32)
            for r in range(self.world):
                BucketIO.unpack(slot[r])  # no-op in bucket-view mode
            self.collectives += 1
            del self._pending[b.index]

    def _finish(self, rank: int) -> None:
        # a rank may finish before its peers submitted; the last rank to finish sees nothing pending
        self._done[rank] = self._done.get(rank, 0) + 1
        if all(self._done.get(r, 0) == self._done[rank] for r in range(self.world)) and self._pending:
            raise RuntimeError(f"virtual ranks finished with buckets {sorted(self._pending)} not reduced on every rank")


class VirtualExecutor(Executor):
    """GradSync executor of one virtual rank (bucket-view mode: grads live in ``b.flat``)."""

    supports_steal = False

    def __init__(self, group: VirtualGroup, rank: int):
        self.group = group
        self.rank = rank

    def submit(self, b) -> None:
        if not b.views:
            from .executor import BucketIO

            BucketIO.pack(b)
        self.group._submit(self.rank, b)

    def finish(self) -> None:
        self.group._finish(self.rank)
