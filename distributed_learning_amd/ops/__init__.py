"""Native (HIP/gfx950) ops and their PyTorch reference fallbacks."""
from . import nn  # noqa: F401
