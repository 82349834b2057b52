"""Whole-training-step HIP graphs.

The reference's step is host-bound Python (data generation on the CPU, two Python threads per
worker spin-waiting on events). Here, once the per-step work is fixed (static
shapes, on-device synthetic data with a device-side stream counter, constant hyper-parameters),
the entire step — data generation, forward, backward with its gradient-ready hooks and the
bucketed RCCL collectives they enqueue on the comm stream, and the fused optimizer — is captured
once into a HIP graph and replayed with a single launch. The ~1-2k kernel launches and the
autograd/Python dispatch of a ResNet-50 step then cost nothing on the host, so the GPU (and the
comm stream) never wait for the CPU.

Capture rules this relies on (and that the framework's ops follow):

* no host synchronisation inside the step (loss stays a device tensor);
* every allocation comes from the caching allocator (the graph's private pool): the C++ ops and
  the comm engine allocate with ``at::empty`` on the capturing or a joined stream;
* side streams join the capture through events (the comm engine's ``join_current`` /
  ``wait_on_current``), so the collectives become graph nodes ordered after the hooks that
  produced their buckets;
* library algorithm selection (MIOpen find, RCCL communicator setup) happens in the eager warmup
  steps before capture.

Gradients live in the graph pool after capture; ``p.grad`` keeps pointing at them, so the captured
optimizer and any inspection between replays see the same storage.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphedStep:
    """``GraphedStep(step_fn)()`` runs ``step_fn`` eagerly for ``warmup`` calls (on a side stream,
    as capture requires), captures the next call, and replays the graph from then on.

    ``step_fn`` must return the step's outputs as device tensors (e.g. the loss); the replayed
    call returns the same (static) tensors, overwritten in place by each replay.
    """

    def __init__(self, step_fn: Callable[[], object], warmup: int = 3, device: Optional[torch.device] = None,
                 enabled: bool = True):
        self.step_fn = step_fn
        self.warmup = max(1, int(warmup))
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.enabled = enabled and self.device.type == "cuda"
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None
        self.calls = 0

    @property
    def captured(self) -> bool:
        return self.graph is not None

    def _capture(self):
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.step_fn()
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.out = self.step_fn()
        self.graph = g

    def __call__(self):
        self.calls += 1
        if not self.enabled:
            return self.step_fn()
        if self.graph is None:
            self._capture()  # capturing records the step without executing it; the replay runs it
        self.graph.replay()
        return self.out

    def reset(self):
        self.graph = None
        self.out = None
