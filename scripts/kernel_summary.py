#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace`` (CSV or rocpd .db) over the steady-state training steps only.

The trace of a bench run also contains start-up work (MIOpen find-mode tuning, warm-up steps)
that dwarfs a training step, so the stock ``kernel_stats.csv`` is useless for step anatomy. Steps
are delimited by the framework's on-device synthetic-data kernel (one Philox ``uniform_kernel``
launch per step); the last ``--steps`` steps are aggregated per kernel and per category.

usage: kernel_summary.py TRACE.csv|TRACE_results.db --steps 8 [--out profiles/NAME]
"""
from __future__ import annotations

import argparse
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_rows import load_rows  # noqa: E402

CATS = [
    ("conv_wgrad", re.compile(r"wrw|bwd_weight|BwdWeight|conv_bwd_w|conv3x3_wgrad|stem_wgrad", re.I)),
    ("conv_dgrad", re.compile(r"igemm_bwd|bwd_data|conv_bwd_d|BwdData|naive_conv.*_bwd|conv3x3(s2)?_dgrad", re.I)),
    ("conv_fwd", re.compile(r"igemm_fwd|conv_fwd|ConvFwd|naive_conv.*_fwd|grouped_conv_fwd|conv3x3_fwd|conv3x3_halo|stem_f", re.I)),
    ("gemm", re.compile(r"gemm|Cijk|dla_gemm|splitk_reduce|conv1x1_dual", re.I)),
    ("batchnorm", re.compile(r"BatchNorm|bn_", re.I)),
    ("dla_bn_act", re.compile(r"bn_act|bnact", re.I)),
    ("optimizer", re.compile(r"sgd_kernel|multi_tensor|foreach", re.I)),
    ("comm", re.compile(r"nccl|rccl|reduce_sum_kernel|pack_kernel|unpack_kernel", re.I)),
    ("loss", re.compile(r"xent|softmax|nll", re.I)),
    ("data", re.compile(r"uniform_kernel|randint_kernel", re.I)),
    ("pool", re.compile(r"pool", re.I)),
    ("elementwise", re.compile(r"elementwise|Functor|threshold|clamp|fill|copy|SubTensor|Tensor", re.I)),
]


def category(name: str) -> str:
    for c, rx in CATS:
        if rx.search(name):
            return c
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--marker", default="uniform_kernel")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    if True:
        for r in load_rows(a.trace):
            grid = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
            wg = r.get("Workgroup_Size_X", "?")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], grid, wg,
                         r.get("LDS_Block_Size", r.get("Lds_Size", "?")), r.get("VGPR_Count", r.get("Arch_VGPR_Count", "?"))))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < a.steps + 1:
        start = marks[0] if marks else 0
        nsteps = max(1, len(marks))
    else:
        start = marks[-a.steps - 1]
        nsteps = a.steps
    end = marks[-1] if len(marks) > a.steps else len(rows)
    win = rows[start:end] if len(marks) > a.steps else rows[start:]
    if len(marks) > a.steps:
        nsteps = a.steps
    per = defaultdict(lambda: [0, 0])
    cat = defaultdict(int)
    busy = 0
    for s, e, n, *_ in win:
        d = e - s
        per[n][0] += 1
        per[n][1] += d
        cat[category(n)] += d
        busy += d
    wall = (win[-1][1] - win[0][0]) if win else 0
    lines = []
    lines.append(f"# Kernel summary: {a.trace}\n")
    lines.append(f"steady-state steps: {nsteps}; GPU wall per step {wall / nsteps / 1e6:.3f} ms; "
                 f"summed kernel time per step {busy / nsteps / 1e6:.3f} ms\n")
    lines.append("\n## By category (ms per step)\n\n| category | ms/step | % |\n|---|---:|---:|")
    for c, d in sorted(cat.items(), key=lambda x: -x[1]):
        lines.append(f"| {c} | {d / nsteps / 1e6:.3f} | {100 * d / max(1, busy):.1f} |")
    lines.append("\n## Top kernels\n\n| kernel | calls/step | ms/step | % |\n|---|---:|---:|---:|")
    for n, (cnt, d) in sorted(per.items(), key=lambda x: -x[1][1])[:40]:
        short = n if len(n) < 110 else n[:107] + "..."
        lines.append(f"| `{short}` | {cnt / nsteps:.1f} | {d / nsteps / 1e6:.3f} | {100 * d / max(1, busy):.1f} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out + ".md", "w") as f:
            f.write(text)
        # step anatomy: every dispatch of the last steady step, in issue order, with its launch shape
        last = [i for i, r in enumerate(win) if a.marker in r[2]]
        one = win[last[-1]:] if last else win
        with open(a.out + "_dispatches.md", "w") as f:
            f.write("| # | kernel | grid (threads) | wg | LDS | VGPR | us |\n|---:|---|---|---:|---:|---:|---:|\n")
            for i, (s0, e0, n, grid, wg, lds, vg) in enumerate(one):
                short = re.sub(r"\(.*", "", n)[:90]
                f.write(f"| {i} | `{short}` | {grid} | {wg} | {lds} | {vg} | {(e0 - s0) / 1e3:.1f} |\n")


if __name__ == "__main__":
    main()
