#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_conv3x3_autograd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3m_tests.log | head; tail -20 gpurun_out/r3m_tests.log; exit 1; }
tail -1 gpurun_out/r3m_tests.log
for p in 2 4 2 4; do
  timeout -k 10 300 python scripts/bench_layers.py --only wgrad --pipe $p --out gpurun_out/r3m_wg_p$p.jsonl > gpurun_out/r3m_wg.log 2>&1 && echo "pipe=$p $(grep '3x3  wgrad' gpurun_out/r3m_wg.log)"
done
for i in 1 2; do timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r3m_b.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/r3m_b.log | head -1; done
