#!/bin/bash
# Round 4, call g08: DUAL_BN extended to stage 2 (Cout 512, W fragments in registers), 3-stage ring for the plain Cout-512 kernel
# -- tests, then interleaved A/B x2 (default / stage 1 only (g07's default) / DUAL_1X1 off) and a kernel trace of the default
set -o pipefail
O=gpurun_out/g08
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm_dual.py \
  tests/test_gpu_bn_epilogue.py tests/test_gpu_layer_parity.py tests/test_gpu_graph.py tests/test_gpu_wgrad_defer.py \
  > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_default.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "from distributed_learning_amd.ops import conv; conv.DUAL_1X1_MAX_COUT = 256" bench.py \
    --steps 15 --warmup 5 >> $O/ab_stage1.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "from distributed_learning_amd.ops import conv; conv.DUAL_1X1 = False" bench.py \
    --steps 15 --warmup 5 >> $O/ab_sep.jsonl 2>> $O/ab.err || exit 1
done
export TMPDIR=/tmp
run 400 rocprofv3 --kernel-trace -d $O/prof -o trace -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || exit 1
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 5 --out $O/ksum > /dev/null || exit 1
python scripts/stream_timeline.py $O/prof/trace_results.db --steps 5 --out $O/timeline.md > /dev/null || exit 1
rm -f $O/prof/trace_results.db
run 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_bench_batch.py > $O/pytest_bs1280.log 2>&1 || exit 1
