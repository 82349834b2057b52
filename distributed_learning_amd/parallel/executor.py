"""Bucket executors: where and when a ready bucket's pack -> reduce -> unpack runs.

The reference overlaps communication with backward using two Python threads per worker (send:
wait bucket event, fuse, ``reducer.put``; receive: ``reducer.get``, unfuse) synchronised by
``threading.Event``s, with the send thread busy-spinning under the GIL
(/root/reference/src/ourdist.py:102-132,28-36). Here the same pipeline is expressed per device:

* :class:`NativeStreamExecutor` (GPU, production): the C++ engine enqueues wait(event) ->
  pack kernel -> RCCL collective -> unpack kernel on its high-priority comm stream straight from
  the autograd hook; ``finish()`` only makes the compute stream wait on the comm stream — the
  CPU never blocks.
* :class:`TorchStreamExecutor` (GPU, torch.distributed collectives on a side stream): same
  stream/event discipline for the Python algorithms of :mod:`.allreduce`.
* :class:`ThreadExecutor` (CPU/Gloo): one background thread drains an ordered queue (the
  reference's send thread, without the spin-wait); ``finish()`` joins the queue.
* :class:`InlineExecutor`: runs in the caller (sequential F / per-tensor modes, tests).
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, Optional

import torch

from .bucketing import Bucket


def _side_pending(device) -> bool:
    from ..ops import conv

    return device.type == "cuda" and conv.side_pending(device)


def _late_wgrads_into(stream, device) -> None:
    from ..ops import conv

    if device.type == "cuda":
        conv.join_into(stream, device)


class BucketIO:
    """Host-side pack/unpack of a bucket for the non-native paths."""

    @staticmethod
    def pack(b: Bucket) -> None:
        if b.views:  # grads already alias the flat buffer
            return
        if b.pack_table is not None:
            b.pack_table.pack(b.flat, 1.0)
            return
        for p, off in zip(b.params, b.offsets):
            g = p.grad
            dst = b.flat[off:off + p.numel()]
            if g is None:
                dst.zero_()
            else:
                dst.copy_(g.reshape(-1))

    @staticmethod
    def unpack(b: Bucket) -> None:
        if b.views:
            return
        if b.pack_table is not None:
            b.pack_table.unpack(b.flat, 1.0)
            return
        for p, off in zip(b.params, b.offsets):
            if p.grad is not None:
                p.grad.view(-1).copy_(b.flat[off:off + p.numel()]) if p.grad.is_contiguous() else \
                    p.grad.copy_(b.flat[off:off + p.numel()].view_as(p.grad))


class Executor:
    def submit(self, bucket: Bucket) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def finish(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def close(self) -> None:
        pass


class NullExecutor(Executor):
    """No communication (single device): buckets are only bookkeeping."""

    def submit(self, b: Bucket) -> None:
        pass

    def finish(self) -> None:
        pass


class InlineExecutor(Executor):
    def __init__(self, reduce_fn: Callable[[torch.Tensor], None]):
        self.reduce_fn = reduce_fn

    def submit(self, b: Bucket) -> None:
        BucketIO.pack(b)
        self.reduce_fn(b.flat)
        BucketIO.unpack(b)

    def finish(self) -> None:
        pass


class ThreadExecutor(Executor):
    """CPU overlap: an ordered worker thread (the reference's send/receive threads in one)."""

    def __init__(self, reduce_fn: Callable[[torch.Tensor], None]):
        self.reduce_fn = reduce_fn
        self.q: "queue.Queue[Optional[Bucket]]" = queue.Queue()
        self.err: Optional[BaseException] = None
        self.pending = 0
        self.cv = threading.Condition()
        self.t = threading.Thread(target=self._run, name="dla-comm", daemon=True)
        self.t.start()

    def _run(self):
        while True:
            b = self.q.get()
            if b is None:
                return
            try:
                if self.err is None:
                    BucketIO.pack(b)
                    self.reduce_fn(b.flat)
                    BucketIO.unpack(b)
            except BaseException as e:  # propagate to the training thread in finish()
                self.err = e
            finally:
                with self.cv:
                    self.pending -= 1
                    self.cv.notify_all()

    def submit(self, b: Bucket) -> None:
        with self.cv:
            self.pending += 1
        self.q.put(b)

    def finish(self) -> None:
        with self.cv:
            while self.pending > 0:
                self.cv.wait()
        if self.err is not None:
            e, self.err = self.err, None
            raise RuntimeError("gradient communication failed") from e

    def close(self) -> None:
        self.q.put(None)
        self.t.join(timeout=10)


class TorchStreamExecutor(Executor):
    """GPU overlap with torch.distributed collectives issued on a dedicated side stream."""

    def __init__(self, reduce_fn: Callable[[torch.Tensor], None], device: torch.device):
        self.reduce_fn = reduce_fn
        self.stream = torch.cuda.Stream(device=device, priority=-1)

    def submit(self, b: Bucket) -> None:
        cur = torch.cuda.current_stream(b.flat.device)
        self.stream.wait_stream(cur)
        _late_wgrads_into(self.stream, b.flat.device)
        with torch.cuda.stream(self.stream):
            BucketIO.pack(b)
            self.reduce_fn(b.flat)
            BucketIO.unpack(b)

    def finish(self) -> None:
        torch.cuda.current_stream().wait_stream(self.stream)


class NativeStreamExecutor(Executor):
    """GPU overlap through the C++ RCCL engine (pack/collective/unpack on its comm stream)."""

    supports_steal = True

    def __init__(self, engine, algorithm: str = "builtin", passthrough: Optional[bool] = None):
        self.engine = engine
        self.algorithm = algorithm
        # one rank: nothing to reduce, gradients stay where autograd put them (tests can force the
        # full gather/reduce/re-point path with passthrough=False)
        self.passthrough = (engine.impl.world() == 1) if passthrough is None else passthrough
        self._join: dict = {}
        # bucket index -> algorithm (parallel/autotune.py: the fastest verified one for that bucket's
        # size); identical on every rank, so the collective sequences still match
        self.per_bucket: dict = {}

    def algorithm_for(self, b: Bucket) -> str:
        return self.per_bucket.get(b.index, self.algorithm)

    def submit(self, b: Bucket) -> None:
        if self.passthrough:
            return
        dev = b.flat.device
        if _side_pending(dev):
            # weight gradients still running on the conv side stream (ops/conv.py WGRAD_DEFER): the engine
            # waits on the current stream, so issue from a stream that has joined both
            j = self._join.get(dev)
            if j is None:
                j = self._join[dev] = torch.cuda.Stream(device=dev)
            j.wait_stream(torch.cuda.current_stream(dev))
            _late_wgrads_into(j, dev)
            with torch.cuda.stream(j):
                self._submit(b)
            return
        self._submit(b)

    def submit_group(self, group) -> None:
        """A fusion-off launch group (grad_sync.LaunchGroup): its buckets keep one collective each, issued
        together (engine.bucket_allreduce_group)."""
        if self.passthrough:
            return
        dev = group.buf.device
        if _side_pending(dev):
            j = self._join.get(dev)
            if j is None:
                j = self._join[dev] = torch.cuda.Stream(device=dev)
            j.wait_stream(torch.cuda.current_stream(dev))
            _late_wgrads_into(j, dev)
            with torch.cuda.stream(j):
                self._submit_group(group)
            return
        self._submit_group(group)

    def _submit_group(self, group) -> None:
        grads, offs = [], []
        for b, start in zip(group.buckets, group.starts):
            for g, o in (getattr(b, "stolen", None) or []):
                grads.append(g)
                offs.append(start + o)
        algo = self.algorithm_for(group.buckets[0])
        self.engine.bucket_allreduce_group(group.buf, group.starts, [b.numel for b in group.buckets], algo, grads, offs)

    def _submit(self, b: Bucket) -> None:
        algo = self.algorithm_for(b)
        stolen = getattr(b, "stolen", None)
        if stolen is not None:
            self.engine.bucket_allreduce_list(b.flat, algo, [g for g, _ in stolen], [o for _, o in stolen])
            return
        table = None if b.views else b.pack_table
        if not b.views and table is None:
            raise RuntimeError("native executor needs grad-as-bucket-view or a native PackTable")
        self.engine.bucket_allreduce(b.flat, algo, True, table)

    def reserve(self, buckets) -> None:
        """Build the engine's plans and size its scratch / IPC windows for these buckets once, at
        setup (collective for IPC algorithms: every rank calls it in the same order)."""
        if self.passthrough:
            return
        groups = {}
        for b in buckets:
            groups.setdefault((self.algorithm_for(b), b.flat.dtype), []).append(b.flat.numel())
        for (algo, dt), sizes in sorted(groups.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
            self.engine.reserve(algo, sizes, dt)

    def reserve_groups(self, groups) -> None:
        """Staging for the fusion-off launch groups (their buffers are reduced as one staged region)."""
        if self.passthrough:
            return
        by = {}
        for g in groups:
            by.setdefault((self.algorithm_for(g.buckets[0]), g.buf.dtype), []).append(g.buf.numel())
        for (algo, dt), sizes in sorted(by.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
            self.engine.reserve(algo, sizes, dt)

    def finish(self) -> None:
        self.engine.wait_on_current()
