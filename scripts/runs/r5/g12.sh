#!/bin/bash
# Round 5, call g12: fused stem weight gradient v2 (B operand as 128-byte contiguous runs, one quad decode per
# thread per k-step) -- numerics, the stem op alone, and its kernel times
set -o pipefail
O=gpurun_out/r5/g12
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u -m pytest tests/test_gpu_stem_bn_fused.py tests/test_gpu_stem.py -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
run 200 python -u scripts/bench_stem.py > $O/stem_fused.jsonl 2> $O/stem.err || { tail $O/stem.err; exit 1; }
cut -c1-200 $O/stem_fused.jsonl
export TMPDIR=/tmp
R=$(pwd)
run 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/stemprof -o s -- python3 $R/scripts/bench_stem.py --iters 10 \
  > $O/stem_prof.log 2>&1 || { tail $O/stem_prof.log; exit 1; }
find /tmp/stemprof -name '*kernel_stats.csv' -exec cp {} $O/stem_kernel_stats.csv \;
cut -d, -f1-4 $O/stem_kernel_stats.csv | cut -c1-160
