#!/usr/bin/env python3
"""MFMA utilisation per kernel from a rocprofv3 ``--pmc`` counter CSV of a bench run.

Counters (one pass): SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe busy cycles summed over all SIMDs),
GRBM_GUI_ACTIVE (GPU-active clock cycles of the dispatch), SQ_WAVES, SQ_BUSY_CYCLES.
Steady-state steps are delimited by the on-device synthetic-data kernel (one ``uniform_kernel``
per training step), as in kernel_summary.py; the last ``--steps`` steps are aggregated.

  util = MFMA_BUSY / (GRBM_GUI_ACTIVE / xcd_div * 1024 SIMDs)

GRBM_GUI_ACTIVE may be summed over the 8 XCDs (rocprofv3 aggregates per-XCD instances);
``xcd_div`` is chosen so the implied clock (GRBM / xcd_div / duration) is a plausible shader clock
(<= 3 GHz) and is reported with the table.

usage: pmc_mfma.py COUNTERS.csv --steps 2 [--out PREFIX]
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict

SIMDS = 256 * 4


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    n = n.replace("void ", "").replace("dla::", "")
    return n[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--marker", default="uniform_kernel")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    disp = {}
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "t0": int(r["Start_Timestamp"]),
                                                        "t1": int(r["End_Timestamp"]), "c": {}})
            d["c"][r["Counter_Name"]] = float(r["Counter_Value"])
    order = sorted(disp)
    marks = [i for i, k in enumerate(order) if a.marker in disp[k]["name"]]
    if len(marks) > a.steps:
        sel = order[marks[-a.steps - 1]:marks[-1]]
        nsteps = a.steps
    else:
        sel, nsteps = order, 1
    per = defaultdict(lambda: [0, 0.0, 0.0, 0.0])  # calls, ns, mfma busy, grbm
    tot = [0.0, 0.0, 0.0]
    for k in sel:
        d = disp[k]
        c = d["c"]
        p = per[short(d["name"])]
        p[0] += 1
        p[1] += d["t1"] - d["t0"]
        p[2] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        p[3] += c.get("GRBM_GUI_ACTIVE", 0.0)
        tot[0] += d["t1"] - d["t0"]
        tot[1] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        tot[2] += c.get("GRBM_GUI_ACTIVE", 0.0)
    ghz_raw = tot[2] / max(1.0, tot[0])
    xcd_div = 8 if ghz_raw > 3.0 else 1
    lines = [f"# MFMA utilisation per kernel ({a.csv})", "",
             f"steady-state steps: {nsteps}; implied shader clock {ghz_raw / xcd_div:.2f} GHz "
             f"(GRBM_GUI_ACTIVE / {xcd_div} / duration); util = SQ_VALU_MFMA_BUSY_CYCLES / "
             f"(GRBM_GUI_ACTIVE / {xcd_div} x {SIMDS} SIMDs). Durations are from the counter run "
             f"(serialised dispatches).", "",
             f"whole step: {tot[0] / nsteps / 1e6:.3f} ms of kernels, MFMA utilisation "
             f"{100 * tot[1] / max(1.0, tot[2] / xcd_div * SIMDS):.1f}%", "",
             "| kernel | calls/step | ms/step | MFMA util % |", "|---|---:|---:|---:|"]
    for n, (cnt, ns, busy, grbm) in sorted(per.items(), key=lambda x: -x[1][1])[:45]:
        util = 100 * busy / max(1.0, grbm / xcd_div * SIMDS)
        lines.append(f"| `{n}` | {cnt / nsteps:.1f} | {ns / nsteps / 1e6:.3f} | {util:.1f} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out + ".md", "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
