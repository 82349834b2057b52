#!/bin/bash
# fused stem BN+ReLU+max-pool forward: fast index decode, branch-free bf16-key compare; tests + benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_stem.py tests/test_gpu_bn_act.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3x_tests.log | head; tail -20 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
bash scripts/gpu_bench_prof.sh r3x || exit 1
grep -E "GPU wall|bn_relu_maxpool_fwd|maxpool" gpurun_out/ksum_r3x.md | head -5
grep -o '"value": [0-9.]*' gpurun_out/bench_r3x.log | head -1
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/r3x_b.log 2>&1 && grep metric gpurun_out/r3x_b.log >> gpurun_out/r3x_records.jsonl && echo "resnet $(grep -o '"value": [0-9.]*' gpurun_out/r3x_b.log | head -1)"; done
timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on > gpurun_out/r3x_g.log 2>&1 && grep metric gpurun_out/r3x_g.log >> gpurun_out/r3x_records.jsonl && echo "gnet $(grep -o '"value": [0-9.]*' gpurun_out/r3x_g.log | head -1)"
