#!/bin/bash
# fused Inception blocks: unit tests, model parity, graph, GoogLeNet bench + profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_inception.py tests/test_gpu_bn_act.py tests/test_gpu_pool.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2o_inc.log 2>&1 || { echo "inception tests failed"; grep -E "Error|assert|FAIL" gpurun_out/r2o_inc.log | head -20; tail -30 gpurun_out/r2o_inc.log; exit 1; }
grep -cE "PASSED" gpurun_out/r2o_inc.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model_parity.py tests/test_gpu_graph.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r2o_parity.log 2>&1 || { echo "parity/graph failed"; grep -E "Error|assert" gpurun_out/r2o_parity.log | head; tail -30 gpurun_out/r2o_parity.log; exit 1; }
grep -E "PASSED|largest" gpurun_out/r2o_parity.log
timeout -k 10 200 python bench.py --model googlenet --batch 128 --steps 20 --warmup 5 > gpurun_out/r2o_gnet128.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2o_gnet128.log || { tail -20 gpurun_out/r2o_gnet128.log; exit 1; }
timeout -k 10 200 python bench.py --model googlenet --batch 128 --steps 20 --warmup 5 --graph on > gpurun_out/r2o_gnet128g.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2o_gnet128g.log || { tail -20 gpurun_out/r2o_gnet128g.log; exit 1; }
timeout -k 10 200 python bench.py --model googlenet --batch 512 --steps 20 --warmup 5 > gpurun_out/r2o_gnet512.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2o_gnet512.log || { tail -20 gpurun_out/r2o_gnet512.log; exit 1; }
bash scripts/gpu_bench_prof.sh r2o_gnet --model googlenet --batch 128 || { echo "prof failed"; exit 1; }
head -45 gpurun_out/ksum_r2o_gnet.md
