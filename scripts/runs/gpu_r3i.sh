#!/bin/bash
# Inception branches on side streams: correctness + A/B (graph and eager)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_inception.py tests/test_gpu_graph.py tests/test_gpu_dp.py "tests/test_gpu_model_parity.py::test_step0_logits_loss_grads_vs_fp32" -x -q --timeout 300 --timeout-method thread > gpurun_out/r3i_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3i_tests.log | head; tail -30 gpurun_out/r3i_tests.log; exit 1; }
tail -1 gpurun_out/r3i_tests.log
for v in 0 1 0 1; do
  DLA_INCEPTION_STREAMS=$v timeout -k 10 200 python bench.py --model googlenet --batch 128 --steps 30 --warmup 5 --graph on > gpurun_out/r3i.log 2>&1 && echo "graph streams=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3i.log | head -1)" || { tail -20 gpurun_out/r3i.log; exit 1; }
done
for v in 0 1; do
  DLA_INCEPTION_STREAMS=$v timeout -k 10 200 python bench.py --model googlenet --batch 512 --steps 20 --warmup 5 > gpurun_out/r3i.log 2>&1 && echo "eager bs512 streams=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3i.log | head -1)"
done
