#!/bin/bash
# one-rank pass-through leaves unused (aux-head) gradients None: graph / DP / CLI tests, GoogLeNet bench + profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dp.py tests/test_gpu_cli.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3o_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3o_tests.log | head; tail -20 gpurun_out/r3o_tests.log; exit 1; }
tail -1 gpurun_out/r3o_tests.log
timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > gpurun_out/r3o_g.log 2>&1 && grep metric gpurun_out/r3o_g.log >> gpurun_out/r3o_records.jsonl && echo "gnet $(grep -o '"value": [0-9.]*' gpurun_out/r3o_g.log | head -1)"
bash scripts/gpu_bench_prof.sh r3o_gnet --model googlenet --batch 128 --graph on || exit 1
grep -E "GPU wall" gpurun_out/ksum_r3o_gnet.md | head -3
grep metric gpurun_out/bench_r3o_gnet.log | grep -o '"value": [0-9.]*' | head -1
