#!/bin/bash
# Round 5, call g37: per-kernel LDS conflicts, waits and instruction mix over the whole step (anonymous-namespace kernels split out)
set -o pipefail
O=gpurun_out/r5/g37
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA \
  SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pc -o c -- python3 $R/bench.py --steps 3 --warmup 2 \
  > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
T=$(find /tmp/pc -name '*counter_collection.csv' | head -1)
python3 - "$T" <<'PY'
import csv, collections, re, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "").replace("dla::", "")[:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "GRBM_GUI_ACTIVE": n[k] += 1
rows = sorted(agg.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"])
with open("gpurun_out/r5/g37/lds_conflicts.md", "w") as f:
    f.write("| kernel | dispatches | GRBM (XCD-summed) | LDS insts | bank-conflict cycles | conflicts / GRBM | VALU / MFMA | wait / wave cycles |\n|---|---:|---:|---:|---:|---:|---:|---:|\n")
    for k, v in rows[:40]:
        g = v["GRBM_GUI_ACTIVE"]
        f.write(f"| `{k}` | {n[k]} | {g:.3g} | {v['SQ_INSTS_LDS']:.3g} | {v['SQ_LDS_BANK_CONFLICT']:.3g} | "
                f"{v['SQ_LDS_BANK_CONFLICT'] / max(g, 1) :.2f} | {v['SQ_INSTS_VALU'] / max(v['SQ_INSTS_MFMA'], 1):.1f} | {v['SQ_WAIT_ANY'] / max(v['SQ_WAVE_CYCLES'], 1):.2f} |\n")
print(open("gpurun_out/r5/g37/lds_conflicts.md").read()[:6000])
PY
