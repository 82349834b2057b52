"""Tracing ranges for rocprofv3 (``--marker-trace``) and a host-side step profiler.

The reference has manual wall-clock timers only. Here every training phase and
every bucket collective can be bracketed by a roctx range (``torch.cuda.nvtx`` maps to roctx on
ROCm builds) when ``DLA_TRACE=1``, so a ``rocprofv3 --marker-trace --kernel-trace`` timeline shows
which kernels belong to which phase/bucket. Off by default: zero cost.
"""
from __future__ import annotations

from .. import knobs
import contextlib
import os

import torch

_ON = knobs.get("TRACE") == "1"


def enabled() -> bool:
    return _ON


def set_enabled(on: bool) -> None:
    global _ON
    _ON = bool(on)


def push(name: str) -> None:
    if _ON and torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)


def pop() -> None:
    if _ON and torch.cuda.is_available():
        torch.cuda.nvtx.range_pop()


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx/roctx naming
    push(name)
    try:
        yield
    finally:
        pop()
