"""Join the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_pmc_bench.sh with the kernel durations:
per kernel name, calls per step, ms per step, HBM-side MB per step and achieved TB/s.
(The last `steps` dispatches of every kernel name are taken as the steady state.)"""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3


def load(c):
    rows = list(csv.DictReader(open(f"{d}/pmcb_{c}/p_counter_collection.csv")))
    out = {}
    for r in rows:
        key = int(r["Dispatch_Id"])
        e = out.setdefault(key, {"name": r["Kernel_Name"], "v": 0.0, "t": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e["v"] += float(r["Counter_Value"])
    return out


f, w = load("FETCH_SIZE"), load("WRITE_SIZE")
# steady state: the last third of dispatches (bench: 3 warmup + 3 timed + profiling tail)
ids = sorted(f)
tail = ids[len(ids) // 2:]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for i in tail:
    n = f[i]["name"]
    short = n.split("(")[0][:90]
    a = agg[short]
    a[0] += 1
    a[1] += f[i]["t"] / 1e6
    a[2] += f[i]["v"] / 1024  # FETCH_SIZE is in KB
    a[3] += (w[i]["v"] / 1024) if i in w else 0.0
nst = max(1, round(len(tail) / max(1, len(ids)) * 6))
tot = sum(a[1] for a in agg.values())
print(f"| kernel | calls | ms | fetch MB | write MB | TB/s |\n|---|---:|---:|---:|---:|---:|")
for k, a in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
    tb = (a[2] + a[3]) / 1e6 / (a[1] / 1e3) if a[1] else 0
    print(f"| `{k}` | {a[0]} | {a[1]:.3f} | {a[2]:.0f} | {a[3]:.0f} | {tb:.2f} |")
print(f"\ntotal kernel ms in window: {tot:.2f}")
