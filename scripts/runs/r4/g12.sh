#!/bin/bash
# Record of a past call: the switch it A/Bs was removed from the sources after measuring slower (profiles/r4/README.md).
# Round 4, call g12: fork form with 64-row tiles -- dual tests, then interleaved A/B x2 (fork off = default / fork
# on with 64-row tiles)
set -o pipefail
O=gpurun_out/g12
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gemm_dual.py > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_default.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "from distributed_learning_amd.ops import conv; conv.DUAL_FORK = True" bench.py \
    --steps 15 --warmup 5 >> $O/ab_fork64.jsonl 2>> $O/ab.err || exit 1
done
