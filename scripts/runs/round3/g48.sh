#!/bin/bash
# Round 3, call 48: per-kernel profile of the final default (ResNet-50, bs1280, late 3x3 wgrads).
set -o pipefail
O=gpurun_out/g48; mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g48prof -o prof -- python3 $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1 || { tail -30 $R/$O/prof.log; exit 1; }
cd $R
grep '"metric"' $O/prof.log | tee $O/bench_line.jsonl
T=$(find /tmp/g48prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 20 --out $O/ksum > /dev/null
S=$(find /tmp/g48prof -name '*kernel_stats.csv' | head -1)
cp "$S" $O/kernel_stats.csv
sed -n 1,30p $O/ksum.md
