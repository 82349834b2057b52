#!/bin/bash
# Round 3, call 30: kernel profile of the current default (late 3x3 weight gradients, SCC-clobber fix).
set -o pipefail
O=gpurun_out/g30; mkdir -p $O
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g30prof -o prof -- python3 $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1 || { tail -30 $R/$O/prof.log; exit 1; }
cd $R
grep -o '"ms_per_step": [0-9.]*' $O/prof.log
T=$(find /tmp/g30prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 20 --out $O/ksum > /dev/null
S=$(find /tmp/g30prof -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
gzip -c "$T" > $O/kernel_trace.csv.gz
head -30 $O/ksum.md
