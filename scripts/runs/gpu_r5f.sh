#!/bin/bash
# per-GPU batch sweep on the current kernels (interleaved, one box), ResNet-50 bf16
set -o pipefail
mkdir -p gpurun_out/r5f
for r in 1 2; do
  for b in 512 768 1024; do
    timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 8 > gpurun_out/r5f/b${b}_r$r.log 2>&1 || { tail -20 gpurun_out/r5f/b${b}_r$r.log; exit 1; }
    echo "batch=$b $(grep -o '"value": [0-9.]*' gpurun_out/r5f/b${b}_r$r.log | head -1) $(grep -o '"peak_mem_gb": [0-9.]*' gpurun_out/r5f/b${b}_r$r.log) $(grep -o '"final_loss": [0-9.]*' gpurun_out/r5f/b${b}_r$r.log)" | tee -a gpurun_out/r5f/sweep.txt
  done
done
