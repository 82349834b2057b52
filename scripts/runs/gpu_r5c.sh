#!/bin/bash
# 256x256 8-wave split-K weight gradients (gemm_tn): tests, per-layer wgrad A/B, whole-step A/B
set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c/gemm_tests.log 2>&1 || { tail -30 gpurun_out/r5c/gemm_tests.log; exit 1; }
tail -1 gpurun_out/r5c/gemm_tests.log
for t in 0 1 0 1; do
  DLA_TN256=$t timeout -k 10 240 python -u scripts/bench_layers.py --only wgrad --out gpurun_out/r5c/wg_tn${t}_$RANDOM.jsonl > gpurun_out/r5c/wg.log 2>&1 || { tail -20 gpurun_out/r5c/wg.log; exit 1; }
done
for i in 1 2; do
  for t in 1 0; do
    DLA_TN256=$t timeout -k 10 300 python bench.py > gpurun_out/r5c/bench_tn${t}_${i}.log 2>&1 || { tail -20 gpurun_out/r5c/bench_tn${t}_${i}.log; exit 1; }
    echo "tn256=$t $(grep -o '"value": [0-9.]*' gpurun_out/r5c/bench_tn${t}_${i}.log | head -1)" | tee -a gpurun_out/r5c/ab.txt
  done
done
