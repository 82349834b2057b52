#!/bin/bash
# 256x256 tiles for the stride-2 3x3 data gradient: conv tests, per-layer A/B, whole-step A/B,
# then the full GPU suite + smoke + bench on the final state
set -o pipefail
mkdir -p gpurun_out/r5o
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5o/conv_tests.log 2>&1 || { tail -40 gpurun_out/r5o/conv_tests.log; exit 1; }
tail -1 gpurun_out/r5o/conv_tests.log
for r in 1 2; do
  for t in 0 1; do
    DLA_TILE256=$t timeout -k 10 240 python -u scripts/bench_layers.py --only dgrad --out gpurun_out/r5o/layers_t${t}_r$r.jsonl > gpurun_out/r5o/layers.log 2>&1 || { tail -20 gpurun_out/r5o/layers.log; exit 1; }
  done
done
grep -h "_first" gpurun_out/r5o/layers_t*_r*.jsonl | grep 3x3 | cut -c1-110
bash scripts/gpu_full.sh
