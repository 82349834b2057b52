#!/bin/bash
# Record of a past call: the switch it A/Bs was removed from the sources after measuring slower (profiles/r4/README.md).
# Round 4, call g18: kernel traces with relu(BN2) normalised on load (LAZY_BN_ACT) and without
set -o pipefail
O=gpurun_out/g18
mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 rocprofv3 --kernel-trace -d $O/prof_lazy -o trace -- python3 bench.py --steps 6 --warmup 3 \
  > $O/prof_lazy.log 2>&1 || exit 1
run 300 rocprofv3 --kernel-trace -d $O/prof_off -o trace -- python3 scripts/ab_call.py \
  "from distributed_learning_amd.ops import conv; conv.LAZY_BN_ACT = False" bench.py --steps 6 --warmup 3 \
  > $O/prof_off.log 2>&1 || exit 1
for m in lazy off; do
  python scripts/kernel_summary.py $O/prof_$m/trace_results.db --steps 5 --out $O/ksum_$m > /dev/null || exit 1
  rm -f $O/prof_$m/trace_results.db
done
