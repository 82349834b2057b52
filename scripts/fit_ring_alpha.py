"""Fit T(S) = a + b*S per (algo, channels) to scripts/vrank_ring_timing.py rows and report the
per-step launch cost alpha = a / steps (the input of parallel/cost_model.py ring_model).

    python scripts/fit_ring_alpha.py profiles/r3/vrank_eager.jsonl [more.jsonl ...]

Least squares over the bucket sizes of each (algo, channels, graph) group; ``steps`` is the
schedule's step count (ring / ring_pipe: 2(N-1); direct: 2). The virtual harness moves the N ranks'
links through one GPU's HBM, so ``b`` is not an xGMI bandwidth; ``a`` is the launch structure's cost.
"""
import collections
import json
import sys


def fit(xs, ys):
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx if sxx else 0.0
    return my - b * mx, b


def steps(algo, world):
    return 2 if algo == "direct" else 2 * (world - 1)


def main(paths):
    groups = collections.defaultdict(list)
    for p in paths:
        for line in open(p):
            if line.strip():
                r = json.loads(line)
                groups[(r["algo"], r["channels"], r.get("graph", False), r["world"])].append(r)
    print("| algo | channels | graph | launches | intercept ms | alpha/step us | slope ms/MiB |")
    print("|---|---:|---|---:|---:|---:|---:|")
    for (algo, ch, graph, world), rows in sorted(groups.items()):
        rows.sort(key=lambda r: r["bucket_mib_fp32"])
        a, b = fit([r["bucket_mib_fp32"] for r in rows], [r["ms"] for r in rows])
        print(f"| {algo} | {ch} | {graph} | {rows[0].get('launches', '')} | {a:.4f} | "
              f"{a * 1e3 / steps(algo, world):.1f} | {b:.4f} |")


if __name__ == "__main__":
    main(sys.argv[1:])
