#!/bin/bash
# Round 5, call g32: what limits the register-staged 128x128 1x1 GEMM (fwd 250880 x 256 x 1024 with statistics,
# 18-22 % MFMA busy): three counter passes over that one shape
set -o pipefail
O=gpurun_out/r5/g32
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
pass() {
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pc -o c -- python3 $R/scripts/gemm_one.py 250880 256 1024 fwd 20 \
    >> $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
  find /tmp/pc -name '*counter_collection.csv' -exec cat {} \; >> $O/pmc_all.csv
  rm -rf /tmp/pc
}
pass SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
pass SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LEVEL_WAVES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE
pass SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(l for l in open("gpurun_out/r5/g32/pmc_all.csv") if not l.startswith('"Correlation_Id"') or True):
    if r.get("Kernel_Name", "").find("gemm_nt_kernel") < 0:
        continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:.4g}  (rows {n[k]})")
PY
