#!/bin/bash
# Round 4, call g07: the consuming BN's backward apply inside the one-pass 1x1 gradient kernel (DUAL_BN)
# -- tests, then interleaved A/B x2 (default / DUAL_BN off / DUAL_1X1 off) and a kernel trace of the default
set -o pipefail
O=gpurun_out/g07
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm_dual.py \
  tests/test_gpu_bn_epilogue.py tests/test_gpu_layer_parity.py tests/test_gpu_graph.py tests/test_gpu_wgrad_defer.py \
  > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_dualbn.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "from distributed_learning_amd.ops import conv; conv.DUAL_BN = False" bench.py \
    --steps 15 --warmup 5 >> $O/ab_dual.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "from distributed_learning_amd.ops import conv; conv.DUAL_1X1 = False" bench.py \
    --steps 15 --warmup 5 >> $O/ab_sep.jsonl 2>> $O/ab.err || exit 1
done
export TMPDIR=/tmp
run 400 rocprofv3 --kernel-trace -d $O/prof -o trace -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || exit 1
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 5 --out $O/ksum > /dev/null || exit 1
python scripts/stream_timeline.py $O/prof/trace_results.db --steps 5 --out $O/timeline.md > /dev/null || exit 1
rm -f $O/prof/trace_results.db
run 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_bench_batch.py > $O/pytest_bs1280.log 2>&1 || exit 1
