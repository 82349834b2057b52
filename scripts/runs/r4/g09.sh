#!/bin/bash
# Record of a past call: the switch it A/Bs was removed from the sources after measuring slower (profiles/r4/README.md).
# Round 4, call g09: stage-2 one-pass 1x1 kernel (plain, no BN) with register-held weights + 3-stage ring vs
# the LDS panel + 2 stages vs no stage-2 one-pass kernel; interleaved A/B x2
set -o pipefail
O=gpurun_out/g09
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gemm_dual.py > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_wreg.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "set_dual_wreg(0)" bench.py --steps 15 --warmup 5 >> $O/ab_panel.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "from distributed_learning_amd.ops import conv; conv.DUAL_1X1_MAX_COUT = 256" bench.py \
    --steps 15 --warmup 5 >> $O/ab_stage1.jsonl 2>> $O/ab.err || exit 1
done
