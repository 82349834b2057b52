#!/bin/bash
# wgrad / dgrad overlap (side stream) restricted to the small-M, wave-quantised layers
set -o pipefail
mkdir -p gpurun_out
for r in 0 25088 100352 0 25088 100352; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --wgrad_overlap_rows $r > gpurun_out/r3k.log 2>&1 && echo "overlap_rows=$r $(grep -o '"value": [0-9.]*' gpurun_out/r3k.log | head -1)"
done
