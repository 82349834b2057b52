#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_inception.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2p_pool.log 2>&1 || { echo "pool tests failed"; grep -E "Error|assert|FAIL" gpurun_out/r2p_pool.log | head -20; tail -30 gpurun_out/r2p_pool.log; exit 1; }
tail -1 gpurun_out/r2p_pool.log
timeout -k 10 200 python bench.py --model googlenet --batch 128 --steps 20 --warmup 5 --graph on > gpurun_out/r2p_gnet128g.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2p_gnet128g.log || { tail -20 gpurun_out/r2p_gnet128g.log; exit 1; }
timeout -k 10 200 python bench.py --model googlenet --batch 128 --steps 20 --warmup 5 > gpurun_out/r2p_gnet128.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r2p_gnet128.log
bash scripts/gpu_bench_prof.sh r2p_gnet --model googlenet --batch 128 --graph on || { echo "prof failed"; exit 1; }
grep -E "GPU wall|maxpool|pool \|" gpurun_out/ksum_r2p_gnet.md | head
