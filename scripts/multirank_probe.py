#!/usr/bin/env python3
"""Multi-rank RCCL check of the native comm engine (run under torchrun).

Every rank fills a rank-distinct buffer, runs each CommEngine algorithm (builtin / ring / direct /
central / rsag) and compares with the exact average; then a PipelinedFusedDP step of ResNet-18 on
rank-distinct data must leave identical parameters on every rank. With fewer GPUs than ranks the
ranks share devices (LOCAL_RANK % device_count), which exercises the full N>1 code path on a
one-GPU box as far as RCCL accepts it.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/multirank_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_learning_amd.parallel import context as ctxmod  # noqa: E402


def main():
    c = ctxmod.init(backend="nccl")
    rank, world, dev = c.rank, c.world_size, c.device
    print(f"rank {rank}/{world} on {dev}", flush=True)
    from distributed_learning_amd.parallel.engine import ALGO_CODES, NativeEngine

    eng = c.engine()
    ok = True
    for n in (1, 7, 1000, 100_003, 4_000_037):
        for dtype in (torch.float32, torch.bfloat16):
            g = torch.Generator(device="cpu").manual_seed(17)
            base = torch.randn(world, n, generator=g)
            want = base.mean(0)
            for algo in sorted(set(ALGO_CODES) - {"ring_gpu"}):
                y = base[rank].to(dev, dtype)
                eng.allreduce(y, algo, True)
                eng.wait_on_current()
                tol = 1e-5 if dtype == torch.float32 else 2e-2
                err = (y.float().cpu() - want).abs().max().item()
                if err > tol * max(1.0, want.abs().max().item()):
                    ok = False
                    print(f"rank {rank}: {algo} n={n} {dtype} max err {err}", flush=True)
    # one DP training step on rank-distinct data: parameters must stay bitwise identical
    from distributed_learning_amd.data import SyntheticBatches
    from distributed_learning_amd.models import resnet18
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.optim import FusedSGD
    from distributed_learning_amd.parallel import PipelinedFusedDP, make_reducer

    dnn.set_backend("native")
    for algo in ("builtin", "ring", "direct"):
        torch.manual_seed(rank)  # different init per rank: the wrapper's broadcast must fix it
        m = resnet18(10).to(dev).to(memory_format=torch.channels_last)
        dnn.bf16_weights(m)
        w = PipelinedFusedDP(m, make_reducer("immediate", algo, native=True), 1 << 20, dev)
        opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, master_weights=True)
        data = SyntheticBatches(16, (3, 32, 32), 10, dev, dtype=torch.bfloat16, seed=5, rank=rank,
                                channels_last=True)
        for _ in range(3):
            x, y = data.next()
            opt.zero_grad(set_to_none=True)
            loss = cross_entropy(w(x), y)
            loss.backward()
            w.sync_gradients()
            opt.step()
        flat = torch.cat([p.detach().float().reshape(-1) for p in m.parameters()])
        allp = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        for r in range(world):
            if not torch.equal(allp[r], allp[0]):
                ok = False
                print(f"rank {rank}: {algo}: parameters of rank {r} differ from rank 0 "
                      f"(max {(allp[r] - allp[0]).abs().max().item()})", flush=True)
        w.cleanup()
    t = torch.tensor([0 if ok else 1], device=dev)
    dist.all_reduce(t)
    if rank == 0:
        print("MULTIRANK_PROBE", "PASS" if int(t) == 0 else "FAIL", f"world={world}", flush=True)
    ctxmod.shutdown()
    sys.exit(0 if int(t) == 0 else 1)


if __name__ == "__main__":
    main()
