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

Transports: every schedule runs on RCCL, or -- ``ipc_`` prefix, or an engine created with
``transport="ipc"`` -- on peer-mapped IPC windows with flag barriers (csrc/comm/ipc.h): pulls
from the peers' HBM (same GPU, or over xGMI). ``:C`` suffix = C ring channels.

Every schedule is a cached Plan (csrc/comm/plan.h); :mod:`.virtual` runs the identical plans for
N virtual ranks inside one process (one GPU or the CPU), which is how the N>1 paths are tested
on a one-GPU box.
"""
from __future__ import annotations

import functools
import os
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


def parse_algo(name: str):
    """``[ipc_]<schedule>[:<channels>]`` -> (schedule, channels, ipc). ``ipc_`` runs the schedule on the
    IPC transport (peer-mapped windows, csrc/comm/ipc.h) instead of RCCL; ``:C`` uses the first C
    edge-disjoint rings of the engine's topology (ring schedules; 0 / absent = all)."""
    base, _, ch = name.partition(":")
    ipc = base.startswith("ipc_")
    if ipc:
        base = base[4:]
    if base not in ALGO_CODES:
        raise ValueError(f"unknown native all-reduce algorithm {name!r}; choose from {sorted(ALGO_CODES)} "
                         "(optionally 'ipc_' prefixed and ':<channels>' suffixed)")
    c = int(ch) if ch else 0
    if not 0 <= c <= 15:
        raise ValueError(f"channel count must be 0..15, got {c}")
    return base, c, ipc


@functools.lru_cache(maxsize=None)
def algo_code(name: str) -> int:
    C = _ext.require()
    base, c, ipc = parse_algo(name)
    return int(getattr(C, ALGO_CODES[base])) | (c << 4) | (256 if ipc else 0)


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

    MAP_ATTEMPTS = 3

    def __init__(self, impl, group, device: torch.device, channels: int, transport: str = "rccl"):
        self.impl = impl
        self.group = group
        self.device = device
        self.channels = channels
        self.transport = transport
        self.stale_mappings = 0  # IPC mappings refused by the nonce check (re-allocated)

    @classmethod
    def create(cls, group=None, device: Optional[torch.device] = None, channels: int = 0,
               local_size: Optional[int] = None, accum_fp32: Optional[bool] = None,
               transport: str = "rccl") -> "NativeEngine":
        """``local_size``: ranks per node for the 2-step algorithms (default ``LOCAL_WORLD_SIZE`` or
        the group size); ``accum_fp32``: reduce bf16 buckets in fp32 (default: on when n > 1).

        ``transport``: ``rccl`` builds the RCCL communicator (``ipc_*`` algorithm names still run
        over peer-mapped windows, mapped on first use); ``ipc`` builds no communicator and runs every
        algorithm over the windows -- several ranks on ONE GPU, which RCCL refuses."""
        C = _ext.require()
        if transport not in ("rccl", "ipc"):
            raise ValueError(f"transport must be 'rccl' or 'ipc', got {transport!r}")
        group = group if group is not None else dist.group.WORLD
        ranks = dist.get_process_group_ranks(group) if group is not dist.group.WORLD else list(
            range(dist.get_world_size()))
        n = len(ranks)
        me = ranks.index(dist.get_rank())
        device = device or torch.device("cuda", torch.cuda.current_device())
        topo = topology(n, channels, local_size)
        if transport == "rccl":
            obj: List[object] = [C.CommEngine.get_unique_id() if me == 0 else None]
            dist.broadcast_object_list(obj, src=ranks[0], group=group)
            uid = obj[0]
        else:
            uid = b""
        impl = C.CommEngine(me, n, uid, device.index, topo["rings"], topo["local_size"], topo["local_rings"],
                            topo["node_rings"])
        impl.set_accum_fp32(n > 1 if accum_fp32 is None else bool(accum_fp32))
        return cls(impl, group, device, len(topo["rings"]), transport)

    def probe_clone(self, timeout_s: float = 30.0) -> "NativeEngine":
        """Collective: a second engine over the same group and topology with its OWN communicator
        (a second ncclCommInitRank) and stream, and a short deadline. The autotuner runs every
        non-builtin candidate here, so a schedule that hangs or raises an async error aborts this
        communicator only -- never the one training uses (engine.cpp wait_stream aborts the
        communicators of the engine that timed out)."""
        e = NativeEngine.create(self.group, self.device, channels=self.channels,
                                local_size=int(self.impl.local_size()), accum_fp32=bool(self.impl.accum_fp32()),
                                transport=self.transport)
        e.set_timeout(timeout_s)
        return e

    def set_timeout(self, seconds: float) -> None:
        """Deadline of this engine's waits and IPC barriers (<= 0: ``DLA_COMM_TIMEOUT_S``)."""
        self.impl.set_timeout(float(seconds))

    # -- setup -------------------------------------------------------------------------------
    def uses_ipc(self, algo: str) -> bool:
        return self.transport == "ipc" or parse_algo(algo)[2]

    def reserve(self, algo: str, sizes, dtype: torch.dtype) -> None:
        """Pre-build the plans of these bucket sizes and size the scratch buffer once (IPC
        algorithms: grow and map every rank's window, a collective call)."""
        self.impl.reserve(algo_code(algo), [int(s) for s in sizes], 1 if dtype == torch.bfloat16 else 0)
        if self.uses_ipc(algo):
            self._map_windows()

    def _map_windows(self, force: bool = False) -> None:
        """Collective: every rank calls it at the same point (the need is deterministic, so all
        ranks agree on whether to grow; it is all-gathered anyway). ``force``: allocate and map a
        new window generation even when the current one is large enough (tests cycle windows)."""
        world = self.impl.world()
        # need AND verified capacity are agreed on: a rank whose last mapping attempt failed reports the
        # capacity it has verified (engine.cpp commits a window only in a clean ipc_open), so every rank
        # takes the same branch even after a failed growth that a caller caught
        mine = (int(self.impl.ipc_need()), int(self.impl.ipc_capacity()))
        both: List[object] = [None] * world
        dist.all_gather_object(both, mine, group=self.group)
        need = max(int(n) for n, _ in both)
        cap = min(int(c) for _, c in both)
        if force:
            need = max(need, int((cap - (1 << 20)) / 1.25), 1 << 16)
        elif need <= cap:
            return
        self.impl.synchronize()  # nothing of mine in flight reads a peer window
        dist.barrier(group=self.group)  # ... nor of any peer's that reads mine
        # every step below is agreed on across ranks before the next, so a rank whose allocation or
        # mapping fails (e.g. peer memory this node cannot map) raises on EVERY rank at the same point
        # instead of leaving the others waiting in a collective.
        #
        # Each new window carries a fresh random nonce that every importer reads back through its
        # mapping (CommEngine.ipc_open). A mapping that shows another nonce is a stale view of an
        # earlier window: pulls through it would read old data and its flag would never advance (the
        # window lifecycle is the leading candidate for the round-4 g23 failure, profiles/r5/g02).
        # All ranks then allocate again -- the superseded
        # windows stay allocated until a verified set exists, so the retry lands on fresh addresses.
        size = int(need * 1.25) + (1 << 20)
        stale: List[str] = []
        for attempt in range(self.MAP_ATTEMPTS):
            nonce = int.from_bytes(os.urandom(8), "little") | 1
            handle, err = None, ""
            try:
                handle = self.impl.ipc_alloc(size, nonce)
            except Exception as e:  # noqa: BLE001
                err = f"ipc_alloc: {e}"
            handles: List[object] = [None] * world
            dist.all_gather_object(handles, (handle, nonce, err), group=self.group)
            errs = [e for _, _, e in handles if e]
            if errs:
                raise RuntimeError("IPC window allocation failed: " + "; ".join(errs))
            bad = ""
            try:
                bad = self.impl.ipc_open([h for h, _, _ in handles], [n for _, n, _ in handles])
            except Exception as e:  # noqa: BLE001
                err = f"ipc_open: {e}"
            flags: List[object] = [None] * world
            dist.all_gather_object(flags, (err, bad), group=self.group)
            errs = [e for e, _ in flags if e]
            if errs:
                raise RuntimeError("IPC window mapping failed: " + "; ".join(errs))
            stale = [f"rank {r}: {b}" for r, (_, b) in enumerate(flags) if b]
            if not stale:
                return
            self.stale_mappings += 1
        raise RuntimeError(f"IPC window mapping stayed stale after {self.MAP_ATTEMPTS} attempts: " + "; ".join(stale))

    def remap_windows(self) -> None:
        """Collective: replace every rank's IPC window by a new generation of the same size."""
        self._map_windows(force=True)

    def ipc_error_info(self) -> Dict[str, int]:
        """The first timed-out IPC barrier's record (error, awaited token, peer flag seen, peer rank),
        the host token counter, the verified window generation and stale mappings refused."""
        keys = ("error", "awaited", "seen", "peer", "host_token", "generation", "stale_refused")
        return dict(zip(keys, (int(v) for v in self.impl.ipc_error_info())))

    def _lazy_reserve(self, algo: str, flat: torch.Tensor) -> None:
        """First use of a size the windows do not hold yet: grow them (collective -- the need is a
        deterministic function of the call sequence, so every rank takes this branch together). The
        steady state issues no host collective."""
        if self.uses_ipc(algo) and self.impl.world() > 1:
            self.impl.reserve(algo_code(algo), [flat.numel()], 1 if flat.dtype == torch.bfloat16 else 0)
            if int(self.impl.ipc_need()) > int(self.impl.ipc_capacity()):
                self._map_windows()

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
        self._lazy_reserve(algo, flat)
        self.impl.allreduce(flat, algo_code(algo), average)

    def bucket_allreduce(self, flat: torch.Tensor, algo: str, average: bool = True, table=None,
                         pack_scale: float = 1.0, unpack_scale: float = 1.0) -> None:
        self._lazy_reserve(algo, flat)
        self.impl.bucket_allreduce(flat, algo_code(algo), average, table, pack_scale, unpack_scale)

    def bucket_allreduce_list(self, flat: torch.Tensor, algo: str, grads, offsets, average: bool = True) -> None:
        """Gather autograd-owned ``grads`` into ``flat`` at ``offsets`` on the comm stream, then reduce."""
        self._lazy_reserve(algo, flat)
        self.impl.bucket_allreduce_list(flat, algo_code(algo), average, list(grads), list(offsets))

    def bucket_allreduce_group(self, group: torch.Tensor, starts, counts, algo: str, grads, offsets,
                               average: bool = True) -> None:
        """Per-tensor collectives of a fusion-off launch group (members are slices of ``group``): one
        gather of ``grads`` at ``offsets`` (group-relative), one staging cast and one RCCL group. IPC schedules
        stage the whole group buffer, so their windows are grown for it first (advisor r5)."""
        self._lazy_reserve(algo, group)
        self.impl.bucket_allreduce_group(group, list(starts), list(counts), algo_code(algo), average, list(grads),
                                         list(offsets))

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

    def discard(self) -> None:
        """Abort this engine's communicators (a failed probe) and drop it without waiting."""
        if self.impl is not None:
            try:
                self.impl.abort()
            finally:
                self.impl = None
