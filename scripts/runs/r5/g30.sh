#!/bin/bash
# Round 5, call g30: halo 3x3 weight gradient, strip DMA issue interleaved with the MFMA steps (branch-free decode)
# -- numerics, the 3x3 shape table, kernel counters
set -o pipefail
O=gpurun_out/r5/g30
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
run() { timeout -k 10 "$1" "${@:2}"; }
run 400 python -u -m pytest tests/test_gpu_halo_wgrad.py tests/test_gpu_conv3x3_autograd.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run 300 python -u scripts/bench_conv_tiles.py > $O/conv_tiles.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
python3 -c "
import json
for l in open('$O/conv_tiles.jsonl'):
    d = json.loads(l); print(d['C'], {k: d[k] for k in ('fwd_auto', 'dgrad_auto', 'wgrad')})
"
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d /tmp/p1 -o c -- python3 $R/scripts/bench_halo_wgrad.py \
  > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
find /tmp/p1 -name '*counter_collection.csv' -exec cp {} $O/p1.csv \;
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open("gpurun_out/r5/g30/p1.csv")):
    if "halo_wgrad" in r["Kernel_Name"]:
        agg["halo_wgrad"][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: f"{x:.4g}" for c, x in v.items()})
PY
rm -f $O/p1.csv
