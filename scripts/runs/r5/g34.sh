#!/bin/bash
# Round 5, call g34: bank conflicts / instruction counts of the 128x128 1x1 GEMM after the swizzled staging layout
set -o pipefail
O=gpurun_out/r5/g34
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d /tmp/pc -o c -- \
  python3 $R/scripts/gemm_one.py 250880 256 1024 fwd 20 > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
find /tmp/pc -name '*counter_collection.csv' -exec cp {} $O/pmc.csv \;
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(float)
for r in csv.DictReader(open("gpurun_out/r5/g34/pmc.csv")):
    if "gemm_nt_kernel" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:.4g}")
PY
rm -f $O/pmc.csv
