#!/bin/bash
# GoogLeNet native coverage: any-C 3x3 convs, ceil-mode fused stem pools, model parity, bench + profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_pool.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2k_conv.log 2>&1 || { echo "conv/pool tests failed"; tail -40 gpurun_out/r2k_conv.log; exit 1; }
tail -1 gpurun_out/r2k_conv.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model_parity.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r2k_parity.log 2>&1 || { echo "parity failed"; grep -E "Error|assert" gpurun_out/r2k_parity.log | head; tail -30 gpurun_out/r2k_parity.log; exit 1; }
grep -E "PASS|largest" gpurun_out/r2k_parity.log | head
timeout -k 10 300 python bench.py --model googlenet --batch 128 --steps 20 --warmup 5 > gpurun_out/r2k_gnet128.log 2>&1 && grep metric gpurun_out/r2k_gnet128.log || { tail -20 gpurun_out/r2k_gnet128.log; exit 1; }
timeout -k 10 300 python bench.py --model googlenet --batch 512 --steps 20 --warmup 5 > gpurun_out/r2k_gnet512.log 2>&1 && grep metric gpurun_out/r2k_gnet512.log || { tail -20 gpurun_out/r2k_gnet512.log; exit 1; }
bash scripts/gpu_bench_prof.sh r2k_gnet --model googlenet --batch 128 || { echo "prof failed"; exit 1; }
head -50 gpurun_out/ksum_r2k_gnet.md
timeout -k 10 200 python -X faulthandler bench.py --model googlenet --batch 128 --steps 5 --warmup 2 --graph on > gpurun_out/r2k_graph.log 2>&1; echo "graph rc=$?"; tail -30 gpurun_out/r2k_graph.log
