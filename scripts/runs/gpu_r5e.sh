#!/bin/bash
# tile configs for the narrow (N = 64 / 128) 3x3 and 1x1 shapes on the current main loops:
# auto vs 256x64 (4 waves stacked along M) vs 256x128 (8 waves, 3-stage) vs 128x128 forced
set -o pipefail
mkdir -p gpurun_out/r5e
for r in 1 2; do
  for t in 0 7 4; do
    timeout -k 10 240 python -u scripts/bench_layers.py --only fwd,dgrad --tile $t --out gpurun_out/r5e/layers_t${t}_r$r.jsonl > gpurun_out/r5e/layers.log 2>&1 || { tail -20 gpurun_out/r5e/layers.log; exit 1; }
  done
done
