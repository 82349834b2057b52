"""Time the engine's ring vs pipelined ring (ring_pipe) schedules for N virtual ranks on one GPU.

Both run their production Plans through the device virtual-rank executor (csrc/comm/vexec.h):
links are device copies on the main stream, reduce kernels on the main stream (ring) or, for the
sub-steps flagged overlap_prev (ring_pipe), on a side stream concurrently with the next sub-step's
copies — the RCCL engine's stream structure. One GPU stands in for N, so absolute times are not
xGMI times; the comparison shows what the overlap buys against the doubled step count.

    python scripts/vrank_ring_timing.py [--world 8] [--channels 7] [--graph] [--out profiles/x.jsonl]

Eagerly the executor is host-bound (N ranks x C channels x steps small copies per call); --graph
captures one all-reduce into a HIP graph and times replays, which leaves the device-side cost.
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
    ap.add_argument("--channels", type=int, default=7)
    ap.add_argument("--out", default=None)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows = []
    for mib in (1, 4, 16, 64):
        n = mib * 1024 * 1024 // 4
        bufs = [torch.randn(n, device=dev) for _ in range(a.world)]
        r = {"world": a.world, "channels": a.channels, "bucket_mib_fp32": mib, "graph": a.graph}
        for algo in ("ring", "ring_pipe"):
            fn = lambda: virtual_allreduce(bufs, algo, channels=a.channels, average=False)  # noqa: E731
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
            r[algo + "_ms"] = round(timeit(fn), 4)
        r["pipe_vs_ring"] = round(r["ring_ms"] / r["ring_pipe_ms"], 3)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
