#!/bin/bash
# Round 3, call 45: per-GPU batch 1024 (default) vs 1280 with the round-3 kernels; 2 interleaved rounds.
set -o pipefail
O=gpurun_out/g45; mkdir -p $O
for i in 1 2; do
  for b in 1024 1280; do
    timeout -k 10 300 python3 bench.py --batch $b --steps 20 --warmup 5 > $O/bench_${b}_$i.log 2>&1 || { tail -30 $O/bench_${b}_$i.log; exit 1; }
    echo "batch=$b $(grep -o '"value": [0-9.]*' $O/bench_${b}_$i.log | head -1) $(grep -o '"peak_mem_gb": [0-9.]*' $O/bench_${b}_$i.log)" | tee -a $O/ab.txt
  done
done
