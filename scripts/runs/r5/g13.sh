#!/bin/bash
# Round 5, call g13: counters of the fused stem weight gradient (which unit limits it): two SQ passes over the
# stem micro-benchmark, plus the list of counters this box offers
set -o pipefail
O=gpurun_out/r5/g13
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL \
  SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d /tmp/p1 -o c -- \
  python3 $R/scripts/bench_stem.py --iters 3 > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
find /tmp/p1 -name '*counter_collection.csv' -exec cp {} $O/p1.csv \;
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM \
  SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d /tmp/p2 -o c -- \
  python3 $R/scripts/bench_stem.py --iters 3 > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
find /tmp/p2 -name '*counter_collection.csv' -exec cp {} $O/p2.csv \;
python3 - <<'PY'
import csv, collections
for f in ("p1", "p2"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f"gpurun_out/r5/g13/{f}.csv")):
        if "stem_wgrad_bn" in r["Kernel_Name"] or "quad_reduce" in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print(f, k, {c: f"{x:.4g}" for c, x in v.items()})
PY
