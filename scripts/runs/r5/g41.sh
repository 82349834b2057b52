#!/bin/bash
# Round 5, call g41: epilogue C staging in unpadded XOR-swizzled rows -- numerics (every epilogue user), GEMM and
# 3x3 tables, step x3, per-kernel conflict table
set -o pipefail
O=gpurun_out/r5/g41
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv3x3.py tests/test_gpu_stem.py tests/test_gpu_conv.py \
  tests/test_gpu_gemm_dual.py tests/test_gpu_bench_batch.py tests/test_gpu_conv3x3_autograd.py tests/test_gpu_bn_epilogue.py \
  -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run 300 python -u scripts/bench_gemm_bs1280.py > $O/gemm.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
run 300 python -u scripts/bench_conv_tiles.py > $O/conv_tiles.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
for i in 1 2 3; do
  run 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
grep metric $O/bench.jsonl | cut -c1-200
sed -e 's#g37#g41#g' scripts/runs/r5/g37.sh > /tmp/g41pmc.sh && bash /tmp/g41pmc.sh > /dev/null && head -24 $O/lds_conflicts.md | cut -d'|' -f2,6
