"""Process-group bootstrap and the per-process distributed context.

Reference: ``init_process`` (/root/reference/src/main.py:303-318) sets MASTER_ADDR, a hard-coded
MASTER_PORT=29501 and GLOO_SOCKET_IFNAME, calls ``dist.init_process_group(backend, rank, size)``
and creates ``size`` two-rank groups for its broadcast-emulated NCCL ring. Here:

* one process per GPU: ``LOCAL_RANK`` selects ``cuda:<local_rank>``;
* backend ``nccl`` (= RCCL on ROCm) for GPU runs, ``gloo`` for CPU runs;
* no pairwise groups — RCCL point-to-point replaces the emulation; the native engine
  (:mod:`.engine`) creates its own RCCL communicator from a unique id shared over the store;
* rendezvous at 127.0.0.1 by default (single node), port overridable.
"""
from __future__ import annotations

from .. import knobs
import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.env import DistEnv, dist_env_from_environ

_CTX: Optional["DistContext"] = None


@dataclass
class DistContext:
    env: DistEnv
    backend: str
    device: torch.device
    _engine: object = None
    _engines: dict = None

    @property
    def rank(self) -> int:
        return self.env.rank

    @property
    def world_size(self) -> int:
        return self.env.world_size

    @property
    def local_rank(self) -> int:
        return self.env.local_rank

    @property
    def local_world_size(self) -> int:
        return self.env.local_world_size

    transport: str = "rccl"
    same_device: bool = False

    def engine(self, local_size: Optional[int] = None, channels: int = 0, transport: Optional[str] = None):
        """The native engine for the WORLD group (created lazily, GPU only).

        ``local_size`` (ranks per node of the 2-step algorithms) and ``channels`` (ring channels)
        are part of the engine's topology; ``transport`` (default: the context's, ``rccl`` unless
        the ranks share one GPU) picks RCCL or the IPC windows; one engine is kept per distinct
        (local_size, channels, transport)."""
        from .engine import NativeEngine, topology

        transport = transport or self.transport
        topo = topology(self.world_size, channels, local_size)
        key = (topo["local_size"], len(topo["rings"]), transport)
        if self._engines is None:
            self._engines = {}
        if key not in self._engines:
            self._engines[key] = NativeEngine.create(dist.group.WORLD, self.device, channels=channels,
                                                     local_size=topo["local_size"], transport=transport)
            if self._engine is None:
                self._engine = self._engines[key]
        return self._engines[key]


def init(backend: Optional[str] = None, rank: Optional[int] = None, world_size: Optional[int] = None,
         master_addr: Optional[str] = None, master_port: Optional[int] = None, device: Optional[str] = None,
         timeout_s: float = 600.0, ifname: Optional[str] = None, same_device: Optional[bool] = None,
         transport: Optional[str] = None) -> DistContext:
    """Initialise (or return) the process-wide distributed context.

    ``same_device`` (default: ``DLA_SAME_DEVICE=1``): every rank uses ``cuda:0`` -- N processes
    sharing one GPU, the way the multi-process data path is exercised on a one-GPU box. RCCL
    refuses that, so the process group is Gloo and the gradient engine uses the IPC transport.
    ``transport`` (default ``DLA_TRANSPORT`` or ``rccl``; ``ipc`` when ``same_device``)."""
    if same_device is None:
        same_device = os.environ.get(knobs.env_name("SAME_DEVICE"), "0") == "1"
    transport = transport or knobs.get("TRANSPORT") or ("ipc" if same_device else "rccl")
    global _CTX
    if _CTX is not None:
        return _CTX
    env = dist_env_from_environ()
    if rank is not None:
        env.rank = int(rank)
    if world_size is not None:
        env.world_size = int(world_size)
        if "LOCAL_WORLD_SIZE" not in os.environ:
            env.local_world_size = env.world_size
        if "LOCAL_RANK" not in os.environ:
            env.local_rank = env.rank % max(1, env.local_world_size)
    if master_addr:
        env.master_addr = master_addr
    if master_port:
        env.master_port = int(master_port)
    if ifname:
        os.environ.setdefault("GLOO_SOCKET_IFNAME", ifname)
    use_gpu = torch.cuda.is_available() if device is None else str(device).startswith("cuda")
    if backend is None:
        backend = "nccl" if use_gpu and not same_device else "gloo"
    if same_device and backend == "nccl" and env.world_size > 1:
        raise ValueError("same_device: RCCL cannot run several ranks on one GPU; use the gloo backend")
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", 0 if same_device else env.local_rank % max(1, ndev))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        if env.world_size == 1 and "MASTER_PORT" not in os.environ and master_port is None:
            env.master_port = _free_port()
        kw = dict(backend=backend, rank=env.rank, world_size=env.world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl" and use_gpu:
            kw["device_id"] = dev
        dist.init_process_group(init_method=f"tcp://{env.master_addr}:{env.master_port}", **kw)
    _CTX = DistContext(env, backend, dev)
    _CTX.transport = transport
    _CTX.same_device = bool(same_device)
    return _CTX


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def get_context() -> DistContext:
    if _CTX is None:
        raise RuntimeError("distributed_learning_amd.init() has not been called")
    return _CTX


def is_initialized() -> bool:
    return _CTX is not None


def shutdown() -> None:
    global _CTX
    if _CTX is not None:
        for e in (_CTX._engines or {}).values():
            e.close()
    if dist.is_initialized():
        try:
            dist.barrier()
        except Exception:
            pass
        dist.destroy_process_group()
    _CTX = None


# Horovod-style accessors ------------------------------------------------------------------------
def rank() -> int:
    return get_context().rank


def size() -> int:
    return get_context().world_size


def local_rank() -> int:
    return get_context().local_rank


def local_size() -> int:
    return get_context().local_world_size
