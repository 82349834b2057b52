#!/bin/bash
# 256x256 8-wave tile: correctness, per-layer A/B vs auto tiles, then the round-end checks
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv3x3.py -x -q -k "tile_configs" --timeout 120 --timeout-method thread > gpurun_out/r5a/tile_tests.log 2>&1 || { tail -30 gpurun_out/r5a/tile_tests.log; exit 1; }
tail -2 gpurun_out/r5a/tile_tests.log
for t in 0 8 0 8; do
  timeout -k 10 240 python -u scripts/bench_layers.py --only fwd,dgrad --tile $t --out gpurun_out/r5a/layers_t${t}_$RANDOM.jsonl > gpurun_out/r5a/layers_t$t.log 2>&1 || { tail -20 gpurun_out/r5a/layers_t$t.log; exit 1; }
done
bash scripts/gpu_full.sh
