#!/bin/bash
# Round 3, call 31: compute step on a high-priority stream (the late weight gradients' side stream yields
# to it) vs the default stream; interleaved, 3 rounds; profile of the prio variant.
set -o pipefail
O=gpurun_out/g31; mkdir -p $O
R=$(pwd)
for i in 1 2 3; do
  for v in 0 1; do
    DLA_COMPUTE_PRIO=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "prio=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
DLA_COMPUTE_PRIO=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g31prof -o prof -- python3 $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1 || { tail -30 $R/$O/prof.log; exit 1; }
cd $R
T=$(find /tmp/g31prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 20 --out $O/ksum > /dev/null
head -8 $O/ksum.md | tail -3; grep "bn_bwd_finalize\|bn_stats_finalize" $O/ksum.md
