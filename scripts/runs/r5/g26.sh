#!/bin/bash
# Round 5, call g26: fused stem weight gradient v6 (8 waves per block, 4 waves per SIMD, 128 VGPRs) -- numerics,
# kernel time and the SQ counter pass
set -o pipefail
O=gpurun_out/r5/g26
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem_bn_fused.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/stemprof -o s -- python3 $R/scripts/bench_stem.py --iters 10 \
  > $O/stem_prof.log 2>&1 || { tail $O/stem_prof.log; exit 1; }
find /tmp/stemprof -name '*kernel_stats.csv' -exec cp {} $O/stem_kernel_stats.csv \;
grep -E "stem_wgrad_bn|quad" $O/stem_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL \
  SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d /tmp/p1 -o c -- \
  python3 $R/scripts/bench_stem.py --iters 3 > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
find /tmp/p1 -name '*counter_collection.csv' -exec cp {} $O/p1.csv \;
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("gpurun_out/r5/g26/p1.csv")):
    if "stem_wgrad_bn" in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: f"{x:.4g}" for c, x in v.items()})
PY
