#!/bin/bash
# Round 5, call g28: the bs1280 step with the v7 fused stem weight gradient (driver command x3) and the
# model-level stem tests
set -o pipefail
O=gpurun_out/r5/g28
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem_bn_fused.py tests/test_gpu_stem.py tests/test_gpu_bench_batch.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
done
grep metric $O/bench.jsonl | cut -c1-200
