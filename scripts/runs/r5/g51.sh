#!/bin/bash
# Round 5, call g51: 3x3 weight gradients on the 2-stage LDS-DMA loop (PIPE 2) by default: conv GPU tests, bench x2
set -o pipefail
O=gpurun_out/r5/g51
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_conv3x3_autograd.py tests/test_gpu_wgrad_defer.py \
  tests/test_gpu_bench_batch.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations 5 > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench.jsonl
