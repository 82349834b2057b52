"""Loader for the native extension ``distributed_learning_amd._C``.

Policy (so GPU runs can never silently pass on an eager fallback):
  * On a machine with a GPU, ``require()`` raises if the extension is missing or fails to load.
  * On CPU-only hosts ``available()`` is simply False and callers use their reference path.
The extension is built in-tree by ``python -m distributed_learning_amd._build`` (or
``__graft_entry__.build()``); set ``DLA_AUTOBUILD=1`` to build on first use.
"""
from __future__ import annotations

from .. import knobs
import os

import torch  # noqa: F401  -- must load torch's HIP runtime/RCCL before _C (same SONAMEs)

_C = None
_ERR: Exception | None = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    try:
        variant = knobs.get("EXT_SO") or None
        if variant:  # A/B runs of a variant build (python -m distributed_learning_amd._build -D ... --out ...)
            import importlib.util
            import sys

            spec = importlib.util.spec_from_file_location("distributed_learning_amd._C", variant)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["distributed_learning_amd._C"] = mod
        else:
            from .. import _C as mod  # type: ignore[attr-defined]

        _C = mod
    except Exception as e:  # pragma: no cover - depends on build state
        if knobs.get("AUTOBUILD") == "1":
            from .. import _build

            _build.build()
            from .. import _C as mod  # type: ignore[attr-defined]

            _C = mod
        else:
            _ERR = e


def available() -> bool:
    _load()
    return _C is not None


def require():
    """Return the native module or raise loudly."""
    _load()
    if _C is None:
        raise RuntimeError(
            "distributed_learning_amd native extension (_C.so) is not built or failed to load: "
            f"{_ERR!r}. Build it with `python -m distributed_learning_amd._build`."
        )
    return _C


def gpu_required() -> bool:
    """True when running on a GPU box, where native kernels are mandatory."""
    return torch.cuda.is_available()
