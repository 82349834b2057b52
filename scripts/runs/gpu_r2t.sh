#!/bin/bash
# per-layer: auto pipeline vs forced register staging (PIPE 0) vs forced LDS-DMA (PIPE 2)
set -o pipefail
mkdir -p gpurun_out
for p in -1 0 2 -1 0; do
  timeout -k 10 300 python scripts/bench_layers.py --pipe $p --out gpurun_out/r2t_layers_p$p.jsonl > gpurun_out/r2t_layers_p$p.log 2>&1 || { tail -20 gpurun_out/r2t_layers_p$p.log; exit 1; }
  echo "pipe=$p"; grep -A8 "conv time" gpurun_out/r2t_layers_p$p.log
done
