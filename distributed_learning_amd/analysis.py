"""Results aggregation and plots (reference: /root/reference/measurements/collect_data.py).

The reference loads ``{cat}_{node}_{dev}_times.csv`` for a set of result folders, groups by
(devices, experiment) and takes the mean, computes ``throughput = 1000 * devices * data_len /
batch_ms`` (collect_data.py:45-48), extrapolates an "Ideal" line from the single-device run, and
draws throughput lines, stacked per-phase latency areas and fusion-size bars (collect_data.py:65-142).

This module reproduces that arithmetic on our (schema-identical) CSVs; plotting uses matplotlib when
it is importable and is skipped otherwise. CLI::

    python -m distributed_learning_amd.analysis results/ --out plots/
"""
from __future__ import annotations

import argparse
import glob
import os
import re
from collections import defaultdict
from typing import Dict, List, Tuple

PHASES = ["get_data", "data2dev", "zero_grad", "forward", "backprop", "sync", "optimizer_step"]
LABELS = {  # collect_data.py:53-63
    "ourdist": "2-step pipelining+fusion", "seq_merge": "2-step fusion", "overlap": "2-step pipelining",
    "central_node_reduce": "2-step central reduce", "ddp": "PyTorch DDP", "onestep_reduce": "1-step pipelining+fusion",
    "onestep_overlap": "onestep_overlap", "onestep_seq_merge": "onestep_seq_merge", "single": "Ideal",
    "onestep_central": "1-step central", "onestep_builtin": "1-step RCCL builtin", "onestep_direct": "1-step direct",
}


def read_times_csv(path: str) -> List[Dict[str, float]]:
    """Parse a ``*_times.csv`` (separator ``", "``; reference reads it with sep=' *, *')."""
    rows = []
    with open(path) as f:
        header = [h.strip() for h in re.split(r" *, *", f.readline().strip())]
        for line in f:
            if not line.strip():
                continue
            vals = [v.strip() for v in re.split(r" *, *", line.strip())]
            row: Dict[str, float] = {"experiment_name": vals[0]}
            for k, v in zip(header[1:], vals[1:]):
                try:
                    row[k] = float(v)
                except ValueError:
                    row[k] = float("nan")
            rows.append(row)
    return rows


def folder_devices(folder: str) -> int:
    """``{experiment}_{total_dev}_{job}`` -> total_dev (reference main.py:324)."""
    m = re.search(r"_(\d+)_[^_/]+/?$", folder.rstrip("/"))
    return int(m.group(1)) if m else 1


def load(folders: List[str], skip_first: int = 0) -> Dict[Tuple[int, str], Dict[str, float]]:
    """Mean per (devices, experiment) over all ranks and batches (collect_data.py:45-48)."""
    acc: Dict[Tuple[int, str], Dict[str, List[float]]] = defaultdict(lambda: defaultdict(list))
    for folder in folders:
        dev = folder_devices(folder)
        for path in glob.glob(os.path.join(folder, "*_times.csv")):
            if path.endswith("_device_times.csv"):
                continue
            for row in read_times_csv(path)[skip_first:]:
                key = (dev, str(row["experiment_name"]))
                for k, v in row.items():
                    if k != "experiment_name":
                        acc[key][k].append(v)
    out = {}
    for key, cols in acc.items():
        mean = {k: sum(v) / len(v) for k, v in cols.items() if v}
        if "batch" in mean and "data_len" in mean and mean["batch"] > 0:
            mean["throughput"] = 1000.0 * key[0] * mean["data_len"] / mean["batch"]
        out[key] = mean
    return out


def with_ideal(data: Dict[Tuple[int, str], Dict[str, float]], devices=(2, 4, 8, 16)):
    """Extrapolate the single-device run x N as "Ideal" (collect_data.py:38-43,99)."""
    single = data.get((1, "single"))
    if single and "throughput" in single:
        for n in devices:
            data[(n, "single")] = dict(single, throughput=single["throughput"] * n)
    return data


def table(data) -> str:
    lines = ["| devices | experiment | img/s | batch ms | " + " | ".join(PHASES) + " |",
             "|---:|---|---:|---:|" + "---:|" * len(PHASES)]
    for (dev, exp), m in sorted(data.items()):
        lines.append(f"| {dev} | {LABELS.get(exp, exp)} | {m.get('throughput', float('nan')):.1f} | "
                     f"{m.get('batch', float('nan')):.2f} | " + " | ".join(f"{m.get(p, 0.0):.2f}" for p in PHASES) + " |")
    return "\n".join(lines)


def plot(data, out_dir: str) -> List[str]:
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        return []
    os.makedirs(out_dir, exist_ok=True)
    files = []
    exps = sorted({e for _, e in data})
    fig, ax = plt.subplots(figsize=(7, 4))
    for e in exps:
        pts = sorted((d, m["throughput"]) for (d, ee), m in data.items() if ee == e and "throughput" in m)
        if pts:
            ax.plot([p[0] for p in pts], [p[1] for p in pts], marker="o", label=LABELS.get(e, e))
    ax.set_xlabel("devices")
    ax.set_ylabel("images / s")
    ax.legend(fontsize=7)
    f = os.path.join(out_dir, "throughput.png")
    fig.savefig(f, dpi=120, bbox_inches="tight")
    files.append(f)
    plt.close(fig)
    for e in exps:  # stacked latency breakdown per experiment (plot_abc)
        pts = sorted((d, m) for (d, ee), m in data.items() if ee == e)
        if not pts:
            continue
        fig, ax = plt.subplots(figsize=(6, 4))
        xs = [d for d, _ in pts]
        other = [m.get("data2dev", 0) + m.get("zero_grad", 0) + m.get("optimizer_step", 0) for _, m in pts]
        ys = [[m.get(p, 0) for _, m in pts] for p in ("get_data", "forward", "backprop", "sync")] + [other]
        ax.stackplot(xs, *ys, labels=["get_data", "forward", "backprop", "sync", "other"])
        ax.set_xlabel("devices")
        ax.set_ylabel("ms / batch")
        ax.legend(fontsize=7, loc="upper left")
        f = os.path.join(out_dir, f"{e}_latency.png")
        fig.savefig(f, dpi=120, bbox_inches="tight")
        files.append(f)
        plt.close(fig)
    return files


def fusion_sweep(folder: str) -> List[Tuple[int, float, float]]:
    """(size_KiB, batch_ms, sync_ms) for a ``fusion_experiment_*`` folder (collect_data.py:78-88)."""
    out = []
    for sub in sorted(glob.glob(os.path.join(folder, "*")), key=lambda p: int(os.path.basename(p)) if
                      os.path.basename(p).isdigit() else -1):
        if not os.path.basename(sub).isdigit():
            continue
        d = load([sub])
        for (_, e), m in d.items():
            if e != "warmup":
                out.append((int(os.path.basename(sub)), m.get("batch", float("nan")), m.get("sync", float("nan"))))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("root", help="results root (folders named {experiment}_{devices}_{job})")
    ap.add_argument("--out", default=None)
    ap.add_argument("--skip_first", type=int, default=0, help="drop the first N batches (warm-up)")
    a = ap.parse_args(argv)
    folders = [p for p in glob.glob(os.path.join(a.root, "*")) if os.path.isdir(p)]
    data = with_ideal(load(folders, a.skip_first))
    print(table(data))
    if a.out:
        for f in plot(data, a.out):
            print("wrote", f)


if __name__ == "__main__":
    main()
