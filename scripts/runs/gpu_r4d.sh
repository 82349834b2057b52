#!/bin/bash
# branch-free window matching in the stem BN+pool backward (quad + PoolDy): tests + ResNet-50 bench + profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_stem.py tests/test_gpu_bn_act.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r4d_tests.log | head; tail -20 gpurun_out/r4d_tests.log; exit 1; }
tail -1 gpurun_out/r4d_tests.log
bash scripts/gpu_bench_prof.sh r4d || exit 1
grep -E "GPU wall|quad" gpurun_out/ksum_r4d.md | cut -c1-140 | head -4
grep -o '"value": [0-9.]*' gpurun_out/bench_r4d.log | head -1
timeout -k 10 120 python scripts/pool_probe.py > gpurun_out/r4d_pool.jsonl 2>&1 && cut -c1-110 gpurun_out/r4d_pool.jsonl | grep hw
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/r4d_b.log 2>&1 && echo "resnet $(grep -o '"value": [0-9.]*' gpurun_out/r4d_b.log | head -1)"; done
timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on > gpurun_out/r4d_g.log 2>&1 && echo "gnet $(grep -o "\"value\": [0-9.]*" gpurun_out/r4d_g.log | head -1)"
