"""Time the engine's P2P schedules for N virtual ranks on one GPU, by channel count.

Every algorithm runs its production Plan through the engine's own issuing code
(csrc/comm/plan_exec.h execute_plan + LocalIssuer): one ring step's links of all ranks and channels
are one multi-lane copy launch (one RCCL group on a real node), its reduces one multi-lane reduce
launch, and ring_pipe's flagged sub-steps put their reduces on the side stream. One GPU stands in
for N, so absolute times are HBM copy times, not xGMI times; the point is the launch structure:
C channels must not cost C times the launches (8.58 ms at 7 channels vs 0.54 ms at 1).

    python scripts/vrank_ring_timing.py [--world 8] [--channels 1,7] [--graph] [--out profiles/x.jsonl]

--graph captures one all-reduce into a HIP graph and times replays (device-side cost only); eager
timing includes the host issue cost, from which the per-step launch overhead (alpha) is fitted.
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_learning_amd.parallel.virtual import virtual_allreduce  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--channels", default="1,7")
    ap.add_argument("--algos", default="ring,ring_pipe,direct")
    ap.add_argument("--mib", default="0.0625,1,4,16,64")
    ap.add_argument("--out", default=None)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows = []
    for mib in [float(x) for x in a.mib.split(",")]:
        n = int(mib * 1024 * 1024) // 4
        bufs = [torch.randn(n, device=dev) for _ in range(a.world)]
        for algo in a.algos.split(","):
            for ch in ([int(c) for c in a.channels.split(",")] if algo.startswith("ring") else [0]):
                launches = virtual_allreduce(bufs, algo, channels=ch, average=False)
                fn = lambda: virtual_allreduce(bufs, algo, channels=ch, average=False)  # noqa: E731
                if a.graph:
                    s = torch.cuda.Stream()
                    s.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s):
                        fn()  # warm the allocator / side stream outside capture
                    torch.cuda.current_stream().wait_stream(s)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        fn()
                    fn = g.replay
                r = {"world": a.world, "algo": algo, "channels": ch, "bucket_mib_fp32": mib, "graph": a.graph,
                     "launches": launches, "ms": round(timeit(fn), 4)}
                rows.append(r)
                print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
