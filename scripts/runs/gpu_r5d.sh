#!/bin/bash
# 256x256 8-wave 3x3 weight gradients: conv tests, per-layer wgrad A/B, whole-step A/B
set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_gemm.py tests/test_gpu_pool.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d/tests.log 2>&1 || { tail -30 gpurun_out/r5d/tests.log; exit 1; }
tail -1 gpurun_out/r5d/tests.log
for t in 0 1 0 1; do
  DLA_TN256=$t timeout -k 10 240 python -u scripts/bench_layers.py --only wgrad --out gpurun_out/r5d/wg_tn${t}_$RANDOM.jsonl > gpurun_out/r5d/wg.log 2>&1 || { tail -20 gpurun_out/r5d/wg.log; exit 1; }
done
for i in 1 2; do
  for t in 1 0; do
    DLA_TN256=$t timeout -k 10 300 python bench.py > gpurun_out/r5d/bench_tn${t}_${i}.log 2>&1 || { tail -20 gpurun_out/r5d/bench_tn${t}_${i}.log; exit 1; }
    echo "tn256=$t $(grep -o '"value": [0-9.]*' gpurun_out/r5d/bench_tn${t}_${i}.log | head -1)" | tee -a gpurun_out/r5d/ab.txt
  done
done
bash scripts/runs/gpu_r5e.sh
