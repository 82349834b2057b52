"""Tensor fusion: greedy gradient bucketing in output-first order.

Reference: ``OurDist._fusion_grouping_gen`` (/root/reference/src/ourdist.py:54-68) walks
``reversed(model.parameters())`` and greedily packs parameters while
``running_bytes + size <= grouping_size``; a bucket always takes at least one parameter (so an
oversize tensor gets its own bucket) and ``grouping_size = 0`` yields one parameter per bucket.
``bucketize`` reproduces that rule exactly (SURVEY.md Appendix B layouts are unit-tested).

MI355X layout: each bucket owns ONE flat device buffer; every gradient slot starts on a 64-element
boundary (256 B for fp32), so the pack/unpack/SGD kernels always take their 16-byte vector path
and gradients can alias the bucket buffer directly (``grad_as_bucket_view``: no pack/unpack copy).

Which cap to use on MI355X is derived, not copied from the reference's 25 MiB: see
:mod:`.cost_model` (collective time on 7 xGMI links vs the backward time left after each bucket
becomes ready).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Iterable, List, Sequence

import torch

ALIGN_ELEMS = 64


def _align(n: int, a: int = ALIGN_ELEMS) -> int:
    return (n + a - 1) // a * a


def fusion_groups(params: Sequence[torch.Tensor], grouping_size: int) -> List[List[torch.Tensor]]:
    """The reference's greedy grouping over ``reversed(params)`` (ourdist.py:54-68)."""
    groups: List[List[torch.Tensor]] = []
    cur: List[torch.Tensor] = []
    running = 0
    for p in reversed(list(params)):
        size = p.element_size() * p.numel()
        if not cur or running + size <= grouping_size:
            cur.append(p)
            running += size
        else:
            groups.append(cur)
            cur = [p]
            running = size
    if cur:
        groups.append(cur)
    return groups


@dataclass
class Bucket:
    index: int
    params: List[torch.Tensor]
    offsets: List[int]           # element offset of each param's slot in the flat buffer
    numel: int                   # sum of param numels (payload)
    padded_numel: int            # flat buffer length (aligned slots)
    flat: torch.Tensor | None = None
    ready: int = 0
    launched: bool = False
    pack_table: object = None    # native PackTable (pack mode on GPU)
    views: List[torch.Tensor] = field(default_factory=list)
    is_ready: List[bool] = field(default_factory=list)  # per parameter, this step

    @property
    def nbytes(self) -> int:
        return self.numel * (self.params[0].element_size() if self.params else 4)

    def reset(self) -> None:
        self.ready = 0
        self.launched = False
        self.is_ready = [False] * len(self.params)


def dtype_fusion_groups(params: Sequence[torch.Tensor], grouping_size: int) -> List[List[torch.Tensor]]:
    """Greedy fusion with one open bucket per dtype (mixed-precision models: bf16 weights + fp32 BN).

    Walks ``reversed(params)`` like the reference; a parameter joins the open bucket of its dtype,
    and a bucket is emitted when it closes, so the list order is the order in which buckets become
    complete during backward. With a single dtype this is exactly :func:`fusion_groups`.
    """
    out: List[List[torch.Tensor]] = []
    open_: dict = {}
    for p in reversed(list(params)):
        size = p.element_size() * p.numel()
        cur = open_.get(p.dtype)
        if cur is None:
            open_[p.dtype] = [[p], size]
        elif cur[1] + size <= grouping_size:
            cur[0].append(p)
            cur[1] += size
        else:
            out.append(cur[0])
            open_[p.dtype] = [[p], size]
    # close the remaining buckets in the order of their last (most recently added) parameter
    order = {id(p): i for i, p in enumerate(reversed(list(params)))}
    for group, _ in sorted(open_.values(), key=lambda g: order[id(g[0][-1])]):
        out.append(group)
    return out


def bucketize(params: Iterable[torch.Tensor], grouping_size: int) -> List[Bucket]:
    params = [p for p in params if p.requires_grad]
    buckets = []
    for i, group in enumerate(dtype_fusion_groups(params, grouping_size)):
        offs, cur = [], 0
        for p in group:
            offs.append(cur)
            cur += _align(p.numel())
        buckets.append(Bucket(i, group, offs, sum(p.numel() for p in group), cur))
    return buckets


def bucket_sizes(buckets: Sequence[Bucket]) -> List[int]:
    return [b.numel for b in buckets]
