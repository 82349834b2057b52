"""Rank/size discovery.

The reference takes rank and size as positional CLI arguments that may be ``envarg://VAR``
indirections resolved from MPI's environment (/root/reference/src/utils.py:20-24,
/root/reference/submit.sh:50). We keep ``envarg://`` and add torchrun's variables
(RANK, WORLD_SIZE, LOCAL_RANK, LOCAL_WORLD_SIZE) and OpenMPI/PMI fallbacks.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

_ENVARG = "envarg://"


def eval_arg(arg: str) -> str:
    """Resolve ``envarg://VAR`` to ``os.environ[VAR]``; other strings pass through."""
    if isinstance(arg, str) and arg.startswith(_ENVARG):
        return os.environ[arg[len(_ENVARG):]]
    return arg


def _first(*names: str, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return v
    return default


@dataclass
class DistEnv:
    rank: int
    world_size: int
    local_rank: int
    local_world_size: int
    master_addr: str
    master_port: int

    @property
    def node_rank(self) -> int:
        return self.rank // max(1, self.local_world_size)

    @property
    def num_nodes(self) -> int:
        return max(1, self.world_size // max(1, self.local_world_size))


def dist_env_from_environ(default_port: int = 29501) -> DistEnv:
    rank = int(_first("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", default=0))
    world = int(_first("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", default=1))
    local_rank = int(_first("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", default=rank))
    local_world = int(_first("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS", default=world))
    addr = _first("MASTER_ADDR", default="127.0.0.1")
    port = int(_first("MASTER_PORT", default=default_port))
    return DistEnv(rank, world, local_rank, local_world, addr, port)
