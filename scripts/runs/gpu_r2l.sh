#!/bin/bash
# ResNet-50 default bench (regression check), then GoogLeNet HIP-graph capture (test + bench)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r2l_r50.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/r2l_r50.log || { tail -20 gpurun_out/r2l_r50.log; exit 1; }
timeout -k 10 300 python -X faulthandler -u -m pytest tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2l_graph_test.log 2>&1 || { echo "graph test failed"; tail -40 gpurun_out/r2l_graph_test.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r2l_graph_test.log
timeout -k 10 200 python -X faulthandler bench.py --model googlenet --batch 128 --steps 20 --warmup 5 --graph on > gpurun_out/r2l_gnet_graph.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2l_gnet_graph.log || { tail -30 gpurun_out/r2l_gnet_graph.log; exit 1; }
timeout -k 10 200 python bench.py --model googlenet --batch 512 --steps 20 --warmup 5 --graph on > gpurun_out/r2l_gnet512_graph.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2l_gnet512_graph.log
