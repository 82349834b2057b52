"""Index-range limits of the native kernels, enforced on the host before anything is launched.

Two ranges bound the hand-written kernels:

* **2^24 pixels** (N*H*W of one conv / pool operand): the implicit-GEMM 3x3 convs, the stem
  (space-to-depth 7x7) and the fused stem BN+ReLU+max-pool decode pixel indices with 24-bit
  multiply-shift divisions (csrc/include/dla_mfma.h ``fdiv``). ResNet-50 at 224x224 reaches it at a
  per-GPU batch of 1338 (1338 * 112 * 112 > 2^24).
* **2 GiB per operand**: the MFMA main loops load through buffer descriptors whose out-of-range
  slots use offset 0x80000000 (``kOOB``), so every operand must span fewer than 2^31 bytes
  (checked again in the C++ bindings, csrc/nn_bindings.cpp ``check_span``).

Crossing either range raises :class:`NativeLimitError` naming the operand; nothing silently falls
back to a different (slower) kernel mid-model and nothing computes with wrapped indices.
"""
from __future__ import annotations

PIXEL_LIMIT = 1 << 24
SPAN_LIMIT = 1 << 31


class NativeLimitError(RuntimeError):
    pass


def pixels_ok(n: int, what: str) -> bool:
    """True, or raises when ``n`` pixels exceed the 24-bit index math of ``what``."""
    if n >= PIXEL_LIMIT:
        raise NativeLimitError(
            f"{what}: {n} pixels >= 2^24, beyond the native kernels' 24-bit index math; lower the per-GPU batch "
            f"(ResNet-50 at 224x224: <= 1337) or run with --kernels torch")
    return True


def span_ok(nbytes: int, what: str) -> bool:
    """True, or raises when one operand would span 2 GiB or more."""
    if nbytes >= SPAN_LIMIT:
        raise NativeLimitError(
            f"{what}: {nbytes} bytes >= 2 GiB, beyond the native kernels' buffer-descriptor range; lower the "
            f"per-GPU batch or run with --kernels torch")
    return True
