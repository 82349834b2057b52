#!/bin/bash
# branch-free generic pool kernels + separable 3x3/s1 forward (strips of 4 or 7): tests, microbenchmark, GoogLeNet A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_inception.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3w_tests.log | head; tail -20 gpurun_out/r3w_tests.log; exit 1; }
tail -1 gpurun_out/r3w_tests.log
for v in 4 7 0; do DLA_POOL3_SEP=$v timeout -k 10 120 python scripts/pool_probe.py > gpurun_out/r3w_pool_$v.jsonl 2>&1 && echo "sep=$v" && cut -c1-120 gpurun_out/r3w_pool_$v.jsonl; done
for v in 4 0 4 0; do
  DLA_POOL3_SEP=$v timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > gpurun_out/r3w_g.log 2>&1 && echo "gnet sep=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3w_g.log | head -1)"
done
