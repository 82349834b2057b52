"""distributed_learning_amd — MI355X-native Horovod-style data-parallel training.

A from-scratch re-design of zdule/distributed_learning for AMD Instinct MI355X (gfx950/CDNA4):
PyTorch-ROCm for the framework layer, hand-written HIP kernels for the gradient path
(multi-tensor pack/unpack, ring reduce, fused SGD-momentum, on-device synthetic data, fused
log-softmax+NLL, fused BN+ReLU(+add)), and a C++ RCCL engine (ring / direct / central / builtin
all-reduce over xGMI) on a dedicated HIP stream, overlapped with backward.

Public API (Horovod-style plus the reference's model-wrapper API)::

    import distributed_learning_amd as dla
    dla.init()
    model = dla.PipelinedFusedDP(model, dla.make_reducer(algorithm="ring", native=True))
    ...
    loss.backward(); model.sync_gradients(); optimizer.step()

or::

    opt = dla.DistributedOptimizer(torch.optim.SGD(...), named_parameters=model.named_parameters())
"""
from __future__ import annotations

import torch  # noqa: F401  -- load torch's HIP runtime and RCCL before the native extension

from . import models, ops, parallel  # noqa: F401
from .parallel import (DistributedOptimizer, HierarchicalReducer, ImmediateReducer, OurDist,  # noqa: F401
                       PerTensorDP, PipelinedFusedDP, SeqDist, SeqMergeDist, SequentialFusedDP, SingleDevice,
                       TorchDDP, WarmupDist, WarmupDP, allgather, allreduce, broadcast, broadcast_optimizer_state,
                       broadcast_parameters, init, local_rank, local_size, make_reducer, rank, shutdown, size)

__version__ = "0.1.0"
