"""Loader for the native extension ``distributed_learning_amd._C``.

Policy (so GPU runs can never silently pass on an eager fallback, or on an old binary):
  * On a machine with a GPU, ``require()`` raises if the extension is missing or fails to load.
  * A binary whose embedded source digest (``_C.source_hash``, written by _build.py) differs from the
    csrc/ tree it runs from is refused (``DLA_ALLOW_STALE=1`` overrides, for debugging).
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

        stale = stale_reason(mod)
        if stale and knobs.get("ALLOW_STALE") != "1":
            raise RuntimeError(stale)
        _C = mod
    except Exception as e:  # pragma: no cover - depends on build state
        if knobs.get("AUTOBUILD") == "1":
            from .. import _build

            _build.build()
            from .. import _C as mod  # type: ignore[attr-defined]

            _C = mod
        else:
            _ERR = e


def stale_reason(mod, root=None) -> str:
    """"" when ``mod`` was built from the csrc/ tree next to this package (the digest _build.py embeds),
    else why not. A tree without csrc/ (an installed copy) is not checked."""
    from pathlib import Path

    from .. import _build

    root = Path(root) if root is not None else Path(_build.ROOT)
    if not (root / "csrc" / "kernels").is_dir():
        return ""
    built = getattr(mod, "source_hash", None)
    if built is None:
        return "the native extension carries no source digest (built before digests existed); rebuild it"
    want = _build.source_digest(root)
    if built != want:
        return (f"stale native extension {getattr(mod, '__file__', '?')}: built from sources {built[:16]}, the tree "
                f"has {want[:16]}; rebuild with `python -m distributed_learning_amd._build`")
    return ""


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
