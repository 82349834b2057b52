"""Data parallelism: bucketing, all-reduce algorithms, reducers, executors, wrappers, optimizer."""
from .allreduce import (ALGORITHMS, Ring, built_in_allreduce, central_allreduce, direct_allreduce,  # noqa: F401
                        edge_disjoint_rings, get_algorithm, ring_allreduce, ring_allreduce_gpu, split_ranges)
from .bucketing import Bucket, bucketize, fusion_groups  # noqa: F401
from .context import DistContext, get_context, init, is_initialized, local_rank, local_size, rank, shutdown, size  # noqa: F401
from .grad_sync import GradSync, find_unused_parameters, make_executor  # noqa: F401
from .optimizer import (DistributedOptimizer, allgather, allreduce, allreduce_, broadcast,  # noqa: F401
                        broadcast_optimizer_state, broadcast_parameters)
from .reducers import (HierarchicalReducer, ImmediateReducer, NativeReducer, ReduceImmediatelly, Reducer,  # noqa: F401
                       make_reducer)
from .wrappers import (OurDist, PerTensorDP, PipelinedFusedDP, SeqDist, SeqMergeDist, SequentialFusedDP,  # noqa: F401
                       SingleDevice, TorchDDP, WarmupDist, WarmupDP, broadcast_module)
