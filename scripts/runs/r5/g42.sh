#!/bin/bash
# Round 5, call g42: the one-pass kBN kernel's in-place BN pass with a conflict-free lane map -- numerics, step x3,
# and the per-kernel counter table
set -o pipefail
O=gpurun_out/r5/g42
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_dual.py tests/test_gpu_bench_batch.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
grep metric $O/bench.jsonl | cut -c1-200
sed -e 's#g37#g42#g' scripts/runs/r5/g37.sh > /tmp/g42pmc.sh && bash /tmp/g42pmc.sh > /dev/null && grep -E "conv1x1_dual" $O/lds_conflicts.md
