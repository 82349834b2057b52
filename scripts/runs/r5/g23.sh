#!/bin/bash
# Round 5, call g23: halo-tiled stem forward v2 (weights in VGPRs, 2 blocks/CU, pipelined A reads) vs the
# implicit GEMM: numerics, the stem op alone x2 each, kernel times, one SQ counter pass of the halo kernel
set -o pipefail
O=gpurun_out/r5/g23
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u -m pytest tests/test_gpu_stem.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  DLA_STEM_HALO=0 run 200 python -u scripts/bench_stem.py >> $O/stem_implicit.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  DLA_STEM_HALO=1 run 200 python -u scripts/bench_stem.py >> $O/stem_halo.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
cut -c1-120 $O/stem_implicit.jsonl $O/stem_halo.jsonl
DLA_STEM_HALO=1 run 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sp -o s -- python3 $R/scripts/bench_stem.py --iters 10 \
  > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
find /tmp/sp -name '*kernel_stats.csv' -exec cp {} $O/stem_kernel_stats_halo.csv \;
grep -E "stem" $O/stem_kernel_stats_halo.csv | cut -d, -f1-4 | cut -c1-140
DLA_STEM_HALO=1 timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL \
  SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d /tmp/p1 -o c -- \
  python3 $R/scripts/bench_stem.py --iters 3 > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
find /tmp/p1 -name '*counter_collection.csv' -exec cp {} $O/p1.csv \;
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("gpurun_out/r5/g23/p1.csv")):
    if "stem_halo" in r["Kernel_Name"] or "stem_fwd" in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: f"{x:.4g}" for c, x in v.items()})
PY
rm -f $O/p1.csv
