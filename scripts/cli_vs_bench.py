"""Compare the reference-compatible CLI's throughput (times.csv through analysis.load, the
reference's collect_data.py arithmetic) with bench.py's JSON line, and with the reference's own
published CSV for the same experiment.

    python scripts/cli_vs_bench.py --cli results/experiment_single_1_x [--bench bench.log]
        [--reference /root/reference/measurements/gpu2/results/experiment_single_1_33846316]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd import analysis  # noqa: E402


def cli_rows(folder):
    data = analysis.load([folder])
    out = {}
    for (dev, exp), row in data.items():
        out[exp] = {"devices": dev, "img_s": round(row["throughput"], 1), "batch_ms": round(row["batch"], 3),
                    **{p: round(row[p], 3) for p in analysis.PHASES if p in row}}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cli", action="append", default=[])
    ap.add_argument("--bench", default=None)
    ap.add_argument("--reference", default=None)
    a = ap.parse_args()
    rec = {}
    for f in a.cli:
        rec[os.path.basename(f.rstrip("/"))] = cli_rows(f)
    if a.bench:
        for line in open(a.bench):
            if line.startswith("{"):
                b = json.loads(line)
                rec["bench"] = {"img_s": b["value"], "ms_per_step": b["ms_per_step"], "config": b["config"]}
    if a.reference and os.path.isdir(a.reference):
        rec["reference"] = cli_rows(a.reference)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
