"""Join the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_pmc_bench.sh with the kernel durations:
HBM-side MB and achieved TB/s per kernel, per step.

    python scripts/pmc_bytes.py [DIR=gpurun_out] [--by-grid]

Steady state: the dispatches between the last-but-``steps`` and the last ``xent_mean_kernel`` (one per
training step), i.e. ``steps`` whole step cycles of the profiled run. ``--stats kernel_stats.csv`` (a
rocprofv3 --stats run without counters) takes each kernel's mean duration from that run instead of
the counter run, whose serialised dispatches are slower. ``--by-grid`` keys the rows by (kernel, grid
size), which separates the layers one GEMM / conv template serves. Durations are those of the counter
run (dispatches serialised by the profiler): within a few % of the kernel-trace run for kernels of
more than ~50 us.
"""
import argparse
import collections
import csv


def load(d, c):
    out = {}
    for r in csv.DictReader(open(f"{d}/pmcb_{c}/p_counter_collection.csv")):
        key = int(r["Dispatch_Id"])
        e = out.setdefault(key, {"name": r["Kernel_Name"], "grid": r.get("Grid_Size", ""), "v": 0.0,
                                 "t": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e["v"] += float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--stats", default="")
    # gfx950: FETCH_SIZE reports half the bytes of streaming reads (a pass reading and writing the same
    # tensor shape, bn_apply_kernel<bf16, false, true, false>, shows fetch = write / 2); scale 2 corrects it
    ap.add_argument("--fetch-scale", type=float, default=1.0)
    a = ap.parse_args()
    f, w = load(a.dir, "FETCH_SIZE"), load(a.dir, "WRITE_SIZE")
    ids = sorted(f)
    marks = [i for i in ids if "xent_mean" in f[i]["name"]]
    steps = min(a.steps, max(1, len(marks) - 1))
    start = marks[-steps - 1] if len(marks) > steps else ids[len(ids) // 2]
    end = marks[-1] if len(marks) > steps else ids[-1]
    tail = [i for i in ids if start < i <= end]
    mean_ns = {}
    if a.stats:
        for r in csv.DictReader(open(a.stats)):
            mean_ns[r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:90]] = float(r["AverageNs"])
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for i in tail:
        short = f[i]["name"].replace("(anonymous namespace)::", "").split("(")[0][:90]
        key = (short, f[i]["grid"]) if a.by_grid else (short, "")
        e = agg[key]
        e[0] += 1
        e[1] += (mean_ns.get(short, f[i]["t"]) if a.stats else f[i]["t"]) / 1e6
        e[2] += f[i]["v"] / 1024 * a.fetch_scale  # FETCH_SIZE / WRITE_SIZE are in KB
        e[3] += (w[i]["v"] / 1024) if i in w else 0.0
    tot_ms = sum(e[1] for e in agg.values()) / steps
    tot_mb = sum(e[2] + e[3] for e in agg.values()) / steps
    grid_col = " grid |" if a.by_grid else ""
    print(f"steady-state steps: {steps}; per step: {tot_ms:.2f} ms of kernels ({'--stats run' if a.stats else 'counter run'}), "
          f"{tot_mb / 1e3:.1f} GB HBM-side, {tot_mb / 1e6 / (tot_ms / 1e3):.2f} TB/s average\n")
    print(f"| kernel |{grid_col} calls/step | ms/step | fetch MB/step | write MB/step | TB/s |")
    print("|---|" + ("---:|" if a.by_grid else "") + "---:|---:|---:|---:|---:|")
    for (k, g), e in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        tb = (e[2] + e[3]) / 1e6 / (e[1] / 1e3) if e[1] else 0.0
        gc = f" {g} |" if a.by_grid else ""
        print(f"| `{k}` |{gc} {e[0] / steps:g} | {e[1] / steps:.3f} | {e[2] / steps:.0f} | {e[3] / steps:.0f} | {tb:.2f} |")


if __name__ == "__main__":
    main()
