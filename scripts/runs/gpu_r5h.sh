#!/bin/bash
# halo-tiled 64->64 3x3 conv: tests, per-layer A/B (DLA_HALO=0 vs default), whole-step A/B
set -o pipefail
mkdir -p gpurun_out/r5h
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5h/tests.log 2>&1 || { tail -40 gpurun_out/r5h/tests.log; exit 1; }
tail -1 gpurun_out/r5h/tests.log
for h in 0 1 0 1; do
  DLA_HALO=$h timeout -k 10 240 python -u scripts/bench_layers.py --only fwd,dgrad --out gpurun_out/r5h/layers_h${h}_$RANDOM.jsonl > gpurun_out/r5h/layers.log 2>&1 || { tail -20 gpurun_out/r5h/layers.log; exit 1; }
done
for i in 1 2; do
  for h in 1 0; do
    DLA_HALO=$h timeout -k 10 300 python bench.py > gpurun_out/r5h/bench_h${h}_${i}.log 2>&1 || { tail -20 gpurun_out/r5h/bench_h${h}_${i}.log; exit 1; }
    echo "halo=$h $(grep -o '"value": [0-9.]*' gpurun_out/r5h/bench_h${h}_${i}.log | head -1)" | tee -a gpurun_out/r5h/ab.txt
  done
done
