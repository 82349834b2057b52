"""Levelled logging with the reference's interface.

Reference: ``print_d(msg, Level)`` with a hard-coded ``VERBOSE_LEVEL = 3`` (DEBUG always on,
3 lines per batch per worker; /root/reference/src/utils.py:5-17). Here the level defaults to INFO
and is settable via ``DLA_VERBOSE`` or :func:`set_verbosity`; messages carry the rank prefix so
multi-process logs stay readable.
"""
from __future__ import annotations

from .. import knobs
import enum
import os
import sys


class Level(enum.IntEnum):
    WARNING = 1
    INFO = 2
    DEBUG = 3


_VERBOSE = int(knobs.get("VERBOSE") or int(Level.INFO))


def set_verbosity(level: int) -> None:
    global _VERBOSE
    _VERBOSE = int(level)


def get_verbosity() -> int:
    return _VERBOSE


def print_d(msg: str, level: Level = Level.INFO) -> None:
    if level <= _VERBOSE:
        rank = os.environ.get("RANK")
        prefix = f"[rank {rank}] " if rank is not None else ""
        print(prefix + str(msg))
        sys.stdout.flush()
