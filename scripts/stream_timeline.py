#!/usr/bin/env python3
"""Per-stream anatomy of the steady-state training steps from a rocprofv3 ``--kernel-trace`` CSV or rocpd .db.

For each HIP stream (rocprofv3 ``Stream_Id``) over the last ``--steps`` steps (delimited by the
on-device data kernel, as scripts/kernel_summary.py): busy time (union of its kernels' intervals),
kernel count, its top kernels, and how much of it overlaps the other streams' busy time. The
streams of a training step are: the compute stream (forward, data gradients, BatchNorm passes),
the late-weight-gradient side stream (ops/conv.py WGRAD_DEFER) and the engine's comm stream
(gather / staging casts / collectives, csrc/comm/engine.cpp). The question it answers: does the
gradient path overlap the compute stream, and what does the comm stream cost while it does.

usage: stream_timeline.py TRACE.csv[.gz]|TRACE_results.db --steps 5 [--out FILE.md]
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_rows import load_rows  # noqa: E402


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append([a, b])
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="uniform_kernel")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    if True:
        for r in load_rows(a.trace):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "?"),
                         r.get("Queue_Id", "?")))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} step markers ({a.marker}) in the trace")
    lo, hi = marks[-(a.steps + 1)], marks[-1]
    t0, t1 = rows[lo][0], rows[hi][0]
    sel = [r for r in rows[lo:hi]]
    by = defaultdict(list)
    names = defaultdict(lambda: defaultdict(float))
    for s, e, n, st, q in sel:
        by[st].append([s, min(e, t1)])
        names[st][n[:90]] += (e - s) / 1e6
    wall = (t1 - t0) / 1e6 / a.steps
    busy = {st: union(v) for st, v in by.items()}
    lines = [f"# Stream timeline: {a.trace}", "",
             f"steady-state steps: {a.steps}; GPU wall per step {wall:.3f} ms", "",
             "| stream | kernels/step | busy ms/step | % of wall | overlapped by other streams, ms/step | top kernels (ms/step) |",
             "|---|---:|---:|---:|---:|---|"]
    order = sorted(busy, key=lambda st: -length(busy[st]))
    for st in order:
        others = union([iv for o in busy if o != st for iv in busy[o]])
        ov = length(intersect(busy[st], others)) / 1e6 / a.steps
        b = length(busy[st]) / 1e6 / a.steps
        top = sorted(names[st].items(), key=lambda kv: -kv[1])[:4]
        tops = "; ".join(f"`{k}` {v / a.steps:.2f}" for k, v in top)
        lines.append(f"| {st} | {len(by[st]) / a.steps:.0f} | {b:.3f} | {100 * b / wall:.1f} | {ov:.3f} | {tops} |")
    allb = union([iv for v in busy.values() for iv in v])
    lines += ["", f"GPU busy (any stream) {length(allb) / 1e6 / a.steps:.3f} ms/step of {wall:.3f}; "
                  f"idle {wall - length(allb) / 1e6 / a.steps:.3f} ms/step"]
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
