#!/bin/bash
# Round 3, call 47: at the batch-1280 default, which late-wgrad mode (3x3 default vs auto vs all) and
# batch 1280 vs 1336 (the stem's 24-bit limit); 2 interleaved rounds.
set -o pipefail
O=gpurun_out/g47; mkdir -p $O
for i in 1 2; do
  for cfg in "3x3 1280" "auto 1280" "all 1280" "3x3 1336"; do
    set -- $cfg
    L=$O/bench_$1_$2_$i.log
    DLA_WGRAD_DEFER=$1 timeout -k 10 300 python3 bench.py --batch $2 --steps 20 --warmup 5 > $L 2>&1 || { tail -30 $L; exit 1; }
    echo "defer=$1 batch=$2 $(grep -o '"value": [0-9.]*' $L | head -1) $(grep -o '"peak_mem_gb": [0-9.]*' $L)" | tee -a $O/ab.txt
  done
done
