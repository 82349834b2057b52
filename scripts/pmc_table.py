#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 --pmc counters from one or more counter_collection CSVs.

  pmc_table.py CSV [CSV ...] [--match SUBSTR]
Prints, per kernel name (shortened) matching SUBSTR: dispatches, mean duration (us), and the
mean of every counter; plus derived ratios when the counters are present.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("dla::", "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="dla::")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for f in a.csv:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "Counter_Name" not in r or a.match not in r["Kernel_Name"]:
                    continue
                k = short(r["Kernel_Name"])
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = sum(dur[k].values()) / max(1, len(dur[k]))
        print(f"== {k}  dispatches/pass={max(len(v) for v in cs.values())}  mean {d:.1f} us")
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.0f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   {c + ' / WAVE_CYCLES':42s} {m[c] / wc:6.3f}")
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_INSTS_LDS" in m:
            print(f"   {'bank conflict cycles / LDS inst':42s} {m['SQ_LDS_BANK_CONFLICT'] / max(1, m['SQ_INSTS_LDS']):6.3f}")


if __name__ == "__main__":
    main()
