#!/bin/bash
# Record of a past call: the switch it A/Bs was removed from the sources after measuring slower (profiles/r4/README.md).
# Round 4, call g11: fork form of the one-pass 1x1 kernel (DUAL_FORK) -- interleaved A/B x2 (default / DUAL_FORK
# off / stage-2 plain kernel on the LDS weight panel) and a kernel trace of the default
set -o pipefail
O=gpurun_out/g11
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_default.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "from distributed_learning_amd.ops import conv; conv.DUAL_FORK = False" bench.py \
    --steps 15 --warmup 5 >> $O/ab_nofork.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u scripts/ab_call.py "set_dual_wreg(0)" bench.py --steps 15 --warmup 5 >> $O/ab_panel.jsonl 2>> $O/ab.err || exit 1
done
export TMPDIR=/tmp
run 400 rocprofv3 --kernel-trace -d $O/prof -o trace -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || exit 1
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 5 --out $O/ksum > /dev/null || exit 1
python scripts/stream_timeline.py $O/prof/trace_results.db --steps 5 --out $O/timeline.md > /dev/null || exit 1
rm -f $O/prof/trace_results.db
