#!/bin/bash
# Round 3, call 34: weight gradients on the 128x128 4-wave tiles (DLA_TN256=0: shorter blocks that leave
# room on a CU) with the late 3x3 weight gradients on vs the 256x256 8-wave tiles; 3 rounds.
set -o pipefail
O=gpurun_out/g34; mkdir -p $O
for i in 1 2 3; do
  for v in 1 0; do
    DLA_TN256=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "tn256=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
