#!/bin/bash
# Round 4, call g04: BN-backward reduction in the dgrad epilogues at the default batch (1280).
#  A/B (interleaved x2): default vs BN_EPILOGUE=stream (only the persistent streaming 1x1 data gradients
#  carry the reduction) vs BN_EPILOGUE=1 (every dgrad); then one rocprofv3 kernel trace per mode;
#  then the per-shape 1x1 GEMM table (scripts/bench_gemm_bs1280.py).
set -o pipefail
O=gpurun_out/g04
mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 "$1" "${@:2}"; }
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_default.jsonl 2>> $O/ab.err || exit 1
  DLA_BN_EPILOGUE=stream run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_stream.jsonl 2>> $O/ab.err || exit 1
done
for m in 0 stream 1; do
  DLA_BN_EPILOGUE=$m run 400 rocprofv3 --kernel-trace -d $O/prof_$m -o trace -- python3 bench.py --steps 6 --warmup 3 \
    > $O/prof_$m.log 2>&1 || exit 1
  python scripts/kernel_summary.py $O/prof_$m/trace_results.db --steps 5 --out $O/ksum_$m > /dev/null || exit 1
  python scripts/stream_timeline.py $O/prof_$m/trace_results.db --steps 5 --out $O/timeline_$m.md > /dev/null || exit 1
  rm -f $O/prof_$m/trace_results.db  # 20+ MB each: the merge-back cap is 64 MiB per call
done
# per-shape bandwidth of the 1x1 GEMMs at bs1280 (targets for the mid-K kernels)
run 300 python -u scripts/bench_gemm_bs1280.py --out $O/gemm_bs1280.jsonl > $O/gemm_bs1280.log 2>&1 || exit 1
