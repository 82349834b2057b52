"""GradSync: bucketed, ordered, overlapped gradient averaging — the engine behind every DP wrapper.

Reference mechanics (/root/reference/src/ourdist.py):
* ``Group`` (13-51): flat buffer per bucket, ``register_hook`` per tensor counting ready grads,
  an ``Event`` when the bucket is complete, ``fuse``/``unfuse`` copies.
* ``OurDist`` (53-178): buckets from ``_fusion_grouping_gen``, send/receive threads, unused
  parameters found by a DFS of the autograd graph at every forward and given
  ``torch.empty_like`` (uninitialised!) grads, ``sync_gradients`` blocks on an Event.

Fixes and MI355X design:
1. ``register_post_accumulate_grad_hook`` instead of ``register_hook``: the reference's hook fires
   *before* AccumulateGrad writes ``.grad`` and papers over it with a spin
   wait. The post-accumulate hook sees the final gradient; the stream event recorded inside it
   orders the comm stream behind the kernel that produced it.
2. Buckets are launched strictly in index order (bucket k only after 0..k-1), so every rank issues
   identical collective sequences regardless of hook timing — a requirement for RCCL.
3. ``grad_as_bucket_view`` (GPU default): each ``param.grad`` *is* a strided view of its bucket's
   flat buffer, so backward accumulates straight into the communication buffer and no pack/unpack
   pass exists at all; averaging happens inside the collective.
4. Unused parameters get zero gradients (not ``empty_like``) — by graph walk when
   ``find_unused_parameters`` (reference semantics), and in any case by ``flush()`` at sync time,
   which zero-fills and launches whatever never became ready, so a missed parameter can never hang
   the job. With one rank and a pass-through executor nothing is reduced, so they keep
   ``grad = None`` (plain-PyTorch semantics; optimizers skip them) and no fill kernels run.
5. No CPU blocking on GPU: ``synchronize()`` = compute stream waits on the comm stream.
6. Local gradient accumulation: backward passes run under :meth:`GradSync.no_sync` leave their
   gradients in place (the next ``prepare()`` does not reset them) and the next synchronised
   backward adds to them before its buckets launch; ``passes_per_step`` > 1 (Horovod's
   ``backward_passes_per_step``) launches a parameter only on its last backward pass.
"""
from __future__ import annotations

from dataclasses import dataclass

from .. import knobs
import contextlib
from typing import Callable, Iterable, List, Optional, Sequence, Set

import torch

from ..ops import _ext
from .bucketing import Bucket, bucketize
from .executor import (Executor, InlineExecutor, NativeStreamExecutor, ThreadExecutor, TorchStreamExecutor)


def same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same element order in memory (strides of size-1 dims ignored), both dense: a gradient can be
    gathered linearly in place of its parameter."""
    if a.shape != b.shape or not is_dense(a):
        return False
    return all(sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()) if n > 1)


def is_dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense in some dimension order (contiguous, channels_last, ...)."""
    dims = sorted((d for d in range(t.dim()) if t.shape[d] != 1), key=lambda d: t.stride(d))
    expect = 1
    for d in dims:
        if t.stride(d) != expect:
            return False
        expect *= t.shape[d]
    return True


def find_unused_parameters(output, params: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    """Parameters not reachable from ``output``'s autograd graph (reference ourdist.py:137-156)."""
    outs = output if isinstance(output, (list, tuple)) else [output]
    seen = set()
    stack = [o.grad_fn for o in outs if isinstance(o, torch.Tensor) and o.grad_fn is not None]
    reached: Set[int] = set()
    for fn in stack:
        seen.add(fn)
    while stack:
        fn = stack.pop()
        var = getattr(fn, "variable", None)
        if var is not None:
            reached.add(id(var))
        for nxt, _ in fn.next_functions:
            if nxt is not None and nxt not in seen:
                seen.add(nxt)
                stack.append(nxt)
    return [p for p in params if p.requires_grad and id(p) not in reached]


# Fusion off (one bucket per tensor, the reference's main_overlap / main_onestep_overlap): per-tensor
# buckets of one dtype form launch groups of at most LAUNCH_GROUP_BYTES / LAUNCH_GROUP_MAX tensors, whose
# members lie within LAUNCH_GROUP_SPAN consecutive buckets (so a group never waits long for its last
# member). Each tensor keeps its own collective; the group shares one event join, gather launch, staging
# cast and RCCL group (engine.cpp bucket_allreduce_group). Groups launch in the order of their last
# member, and the grouping is a pure function of the parameter list, so every rank issues the same
# sequence. A tensor above the byte cap is a group of its own.
LAUNCH_GROUP_BYTES = 1 << 20
LAUNCH_GROUP_MAX = 16
LAUNCH_GROUP_SPAN = 24


@dataclass
class LaunchGroup:
    buckets: List[Bucket]
    starts: List[int]       # element offset of each bucket's flat buffer in ``buf``
    buf: torch.Tensor = None


def launch_groups(buckets: Sequence[Bucket], max_bytes: int = LAUNCH_GROUP_BYTES, max_tensors: int = LAUNCH_GROUP_MAX,
                  span: int = LAUNCH_GROUP_SPAN, key=None) -> List[List[Bucket]]:
    """Greedy grouping of buckets in index (backward) order, per dtype and per ``key(bucket)`` (the executor's
    algorithm for the bucket: a group runs ONE algorithm for all members, so members never mix schedules whose
    plans / IPC windows were sized for another); returned in launch order (by the index of each group's last
    bucket)."""
    done: List[List[Bucket]] = []
    open_: dict = {}
    for pos, b in enumerate(buckets):
        dt = (b.params[0].dtype, key(b) if key is not None else None)
        nb = b.padded_numel * b.params[0].element_size()
        cur = open_.get(dt)
        if cur is not None:
            members, size, first = cur
            if size + nb > max_bytes or len(members) >= max_tensors or pos - first >= span:
                done.append(members)
                cur = None
        if cur is None:
            open_[dt] = [[b], nb, pos]
        else:
            cur[0].append(b)
            cur[1] += nb
    done.extend(v[0] for v in open_.values())
    pos_of = {id(b): i for i, b in enumerate(buckets)}
    return sorted(done, key=lambda g: pos_of[id(g[-1])])


class GradSync:
    """Owns buckets, hooks and an executor for a fixed parameter list."""

    def __init__(self, params: Iterable[torch.Tensor], *, bucket_cap_bytes: int = 25 * 1024 * 1024,
                 executor: Executor, overlap: bool = True, grad_as_bucket_view: Optional[bool] = None,
                 comm_dtype: Optional[torch.dtype] = None, grad_mode: Optional[str] = None,
                 passes_per_step: int = 1):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("GradSync: no parameters require grad")
        self.device = self.params[0].device
        self.executor = executor
        self.overlap = overlap
        # Gradient storage modes:
        #   "steal" (native engine default): .grad is None before backward, AccumulateGrad hands the
        #           autograd-produced tensor over without a copy; each complete bucket is gathered into
        #           its flat buffer on the comm stream (one by-value multi-tensor launch) and reduced;
        #           after sync every .grad is re-pointed at its averaged slot. No memset, no
        #           accumulate-add kernels. With world size 1 the gradients pass through untouched.
        #   "view": .grad is a persistent view of the bucket buffer (zeroed each step; autograd adds).
        #   "pack": persistent .grad tensors packed/unpacked by a device-table kernel.
        if grad_mode is None:
            if getattr(executor, "supports_steal", False) and (comm_dtype is None) and grad_as_bucket_view is None:
                grad_mode = "steal"
            else:
                grad_mode = None
        self.grad_mode = grad_mode
        # comm_dtype=None: every bucket communicates in its parameters' dtype (mixed-precision
        # models get separate bf16 / fp32 buckets); a dtype here forces a wire format (e.g. bf16
        # compression of fp32 gradients, Horovod's Compression.fp16 analogue).
        self.comm_dtype = comm_dtype
        if grad_as_bucket_view is None:
            grad_as_bucket_view = comm_dtype is None or all(p.dtype == comm_dtype for p in self.params)
        if grad_as_bucket_view and comm_dtype is not None and any(p.dtype != comm_dtype for p in self.params):
            raise ValueError("grad_as_bucket_view requires comm_dtype == parameter dtype")
        self.grad_as_bucket_view = grad_as_bucket_view
        self.buckets: List[Bucket] = bucketize(self.params, bucket_cap_bytes)
        self._owner = {}
        # fusion off on the native engine: per-tensor buckets launched in groups (see LaunchGroup)
        self.groups: List[LaunchGroup] = []
        if grad_mode == "steal":
            self._build_groups()
        for b in self.buckets:
            if b.flat is None:
                b.flat = torch.zeros(b.padded_numel, dtype=comm_dtype or b.params[0].dtype, device=self.device)
            for j, p in enumerate(b.params):
                self._owner[id(p)] = (b, j)
        self._persistent_grads = {}
        self.passthrough = bool(getattr(executor, "passthrough", False))
        if self.grad_mode == "steal":
            self.grad_as_bucket_view = False
            self._install_views(install=False)
            for b in self.buckets:
                b.stolen = []
        elif self.grad_as_bucket_view:
            self.grad_mode = "view"
            self._install_views()
        elif self.device.type == "cuda":
            self.grad_mode = "pack"
            self._install_pack_tables()
        else:
            self.grad_mode = "pack"
        self._next = 0
        self._enabled = True
        self._accum_pending = False  # gradients of no_sync passes are waiting for the synced pass
        if passes_per_step < 1:
            raise ValueError("passes_per_step must be >= 1")
        self.passes_per_step = int(passes_per_step)
        self._pass_count = {}
        self._hooks = []
        # DLA_HOOK_TIMING=1: host seconds spent inside the gradient-ready hooks (the Python work the
        # autograd thread does per parameter, incl. the engine's enqueue of complete buckets)
        self.hook_s, self.hook_calls = 0.0, 0
        if overlap:
            import os

            hook = self._on_grad_ready_timed if knobs.get("HOOK_TIMING") == "1" else self._on_grad_ready
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(hook))
        self.step_count = 0
        if hasattr(self.executor, "reserve"):
            self.executor.reserve(self.buckets)
            if self.groups and hasattr(self.executor, "reserve_groups"):
                self.executor.reserve_groups(self.groups)

    # -------------------------------------------------------------------------------------------
    # setup
    # -------------------------------------------------------------------------------------------
    def _wants_groups(self) -> bool:
        ex = self.executor
        per_tensor = len(self.buckets) > 1 and all(len(b.params) == 1 for b in self.buckets)
        # DLA_LAUNCH_GROUPS=0: strict fusion off -- every tensor its own collective launch, as the reference
        return (knobs.flag("LAUNCH_GROUPS") and per_tensor and self.comm_dtype is None and self.overlap and self.device.type == "cuda"
                and getattr(ex, "supports_steal", False) and hasattr(ex, "submit_group")
                and not getattr(ex, "passthrough", False))

    def _build_groups(self) -> None:
        self.groups = []
        for b in self.buckets:
            b.group = None
        if not self._wants_groups():
            return
        algo_for = getattr(self.executor, "algorithm_for", None)
        for members in launch_groups(self.buckets, key=algo_for):
            starts, n = [], 0
            for b in members:
                starts.append(n)
                n += b.padded_numel
            g = LaunchGroup(members, starts, torch.zeros(n, dtype=members[0].params[0].dtype, device=self.device))
            for b, st in zip(members, starts):
                b.flat = g.buf[st:st + b.padded_numel]
                b.group = g
            self.groups.append(g)

    def set_executor(self, executor: Executor) -> None:
        """Replace the executor after construction (e.g. a forced full data path at one rank); the
        fusion-off launch groups and the steal-mode views follow the new executor."""
        self.executor = executor
        self.passthrough = bool(getattr(executor, "passthrough", False))
        if self.grad_mode == "steal":
            had = bool(self.groups)
            self._build_groups()
            if had or self.groups:
                for b in self.buckets:
                    if b.group is None:
                        b.flat = torch.zeros(b.padded_numel, dtype=b.params[0].dtype, device=self.device)
                self._install_views(install=False)
        if hasattr(executor, "reserve"):
            executor.reserve(self.buckets)
            if self.groups and hasattr(executor, "reserve_groups"):
                executor.reserve_groups(self.groups)
    def regroup(self) -> None:
        """Rebuild the fusion-off launch groups and re-reserve after the executor's per-bucket algorithms were
        set (the autotuner runs after construction; a group must not span two algorithms)."""
        self.set_executor(self.executor)

    def _install_views(self, install: bool = True):
        for b in self.buckets:
            b.views = []
            for p, off in zip(b.params, b.offsets):
                if not is_dense(p):
                    raise ValueError("bucket views need dense parameters")
                v = b.flat[off:off + p.numel()].as_strided(p.shape, p.stride())
                b.views.append(v)
                if install:
                    p.grad = v

    def _install_pack_tables(self):
        """Persistent grad tensors + one native PackTable per bucket (GPU pack mode)."""
        C = _ext.require()
        for b in self.buckets:
            grads = []
            for p in b.params:
                g = torch.zeros_like(p)
                self._persistent_grads[id(p)] = g
                p.grad = g
                grads.append(g)
            b.pack_table = C.PackTable(grads, b.offsets)

    # -------------------------------------------------------------------------------------------
    # per-step protocol
    # -------------------------------------------------------------------------------------------
    def prepare(self) -> None:
        """Call before backward (the wrappers do it in forward): reset counters, zero buffers.

        After backward passes under :meth:`no_sync` the gradients are kept (only the bucket
        counters reset), so the next backward accumulates onto them."""
        self._next = 0
        for b in self.buckets:
            b.reset()
        if self._accum_pending:
            if self.grad_mode == "steal":
                for b in self.buckets:
                    b.stolen = []
            return
        self._pass_count = {}
        if self.grad_mode == "steal":
            for p in self.params:
                p.grad = None
            for b in self.buckets:
                b.stolen = []
        elif self.grad_as_bucket_view:
            for b in self.buckets:
                for p, v in zip(b.params, b.views):
                    if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                        p.grad = v
                b.flat.zero_()
        elif self._persistent_grads:
            for p in self.params:
                g = self._persistent_grads[id(p)]
                if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                    p.grad = g
                g.zero_()
        else:
            for p in self.params:
                if p.grad is not None:
                    p.grad.zero_()

    def mark_ready(self, params: Iterable[torch.Tensor]) -> None:
        """Mark parameters that will receive no gradient (unused) as ready with zero grads."""
        if not self._enabled:
            return
        for p in params:
            if p.grad is None and not self.passthrough:  # one rank: left None (see flush)
                p.grad = torch.zeros_like(p)
            self._ready(p)

    def _on_grad_ready_timed(self, p: torch.Tensor) -> None:
        import time

        t0 = time.perf_counter()
        self._on_grad_ready(p)
        self.hook_s += time.perf_counter() - t0
        self.hook_calls += 1

    def _on_grad_ready(self, p: torch.Tensor) -> None:
        if not self._enabled:
            return
        if self.passes_per_step > 1:
            c = self._pass_count.get(id(p), 0) + 1
            self._pass_count[id(p)] = c
            if c % self.passes_per_step:
                return  # accumulate locally; the last pass of the step launches
        b, j = self._owner[id(p)]
        if self.grad_as_bucket_view and p.grad.data_ptr() != b.views[j].data_ptr():
            # the user replaced .grad (e.g. set_to_none between prepare and backward): fold it back
            if p.grad.is_cuda:  # a late weight gradient (ops/conv.py WGRAD_DEFER) may still be running
                from ..ops import conv as _conv

                _conv.join_into(torch.cuda.current_stream(p.grad.device), p.grad.device)
            b.views[j].copy_(p.grad)
            p.grad = b.views[j]
        self._ready(p)

    def _ready(self, p: torch.Tensor) -> None:
        b, j = self._owner[id(p)]
        if len(b.is_ready) != len(b.params):
            b.is_ready = [False] * len(b.params)
        if b.is_ready[j]:
            raise RuntimeError(f"bucket {b.index}: parameter reported ready twice in one step "
                               "(backward called twice without prepare()/no_sync?)")
        b.is_ready[j] = True
        if self.grad_mode == "steal" and p.grad is not None:
            g = p.grad
            if g.dtype != b.flat.dtype or not same_layout(g, p):
                if g.is_cuda:  # the conversion reads g on the compute stream: wait for a late weight gradient
                    from ..ops import conv as _conv

                    _conv.join_into(torch.cuda.current_stream(g.device), g.device)
                g = g.to(b.flat.dtype) if same_layout(g, p) else torch.empty_like(p, dtype=b.flat.dtype).copy_(g)
            b.stolen.append((g, b.offsets[j]))
        b.ready += 1
        self._launch_in_order()

    def _launch_in_order(self) -> None:
        if self.groups:
            self._launch_groups_in_order()
            return
        while self._next < len(self.buckets) and self.buckets[self._next].ready == len(self.buckets[self._next].params):
            b = self.buckets[self._next]
            b.launched = True
            self._next += 1
            self.executor.submit(b)

    def _launch_groups_in_order(self) -> None:
        # self._next counts groups (in launch order); a group goes out when all of its buckets are ready
        # and every earlier group has gone out
        while self._next < len(self.groups):
            g = self.groups[self._next]
            if any(b.ready != len(b.params) for b in g.buckets):
                return
            for b in g.buckets:
                b.launched = True
            self._next += 1
            self.executor.submit_group(g)

    def flush(self) -> None:
        """Launch every bucket that has not been launched (zero-filling missing grads).

        One rank with a pass-through executor reduces nothing, so parameters that got no gradient
        (GoogLeNet's unused aux heads) keep ``grad = None`` as in plain PyTorch, and optimizers skip
        them, instead of paying a zero-fill launch per tensor every step."""
        for b in [b for b in self.buckets if not b.launched]:
            if b.ready < len(b.params):
                if self.grad_mode == "steal":
                    if len(b.is_ready) != len(b.params):
                        b.is_ready = [False] * len(b.params)
                    for j, p in enumerate(b.params):
                        if not b.is_ready[j]:  # (marked-unused parameters are ready already)
                            if p.grad is None and not self.passthrough:
                                p.grad = torch.zeros_like(p)
                            self._ready(p)  # records the gradient (no launch: bucket incomplete until the end)
                else:
                    for p in b.params:
                        if p.grad is None and not self.passthrough:
                            p.grad = torch.zeros_like(p)
                b.ready = len(b.params)
        self._launch_in_order()

    def synchronize(self) -> None:
        """All buckets reduced; the caller's stream (GPU) / thread (CPU) may use the grads."""
        if not self._enabled:
            return
        self.flush()
        self.executor.finish()
        if self.grad_mode == "steal" and not self.passthrough:
            for b in self.buckets:
                for p, v in zip(b.params, b.views):
                    p.grad = v
                b.stolen = []  # autograd's tensors are released only after the compute stream joined
        self._accum_pending = False
        self._pass_count = {}
        self.step_count += 1

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (hooks do not communicate) inside this context; the next
        synchronised backward adds to them and reduces the sum."""
        prev = self._enabled
        self._enabled = False
        try:
            yield
        finally:
            self._enabled = prev
            self._accum_pending = True

    def close(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.executor.close()


# ---------------------------------------------------------------------------------------------
# executor selection
# ---------------------------------------------------------------------------------------------
def make_executor(reducer, device: torch.device, overlap: bool = True) -> Executor:
    """Pick the executor for a reducer on a device (see executor.py)."""
    if getattr(reducer, "native", False):
        return NativeStreamExecutor(reducer.engine, reducer.algorithm)
    if device.type == "cuda":
        return TorchStreamExecutor(reducer.reduce, device)
    if overlap:
        return ThreadExecutor(reducer.reduce)
    return InlineExecutor(reducer.reduce)
