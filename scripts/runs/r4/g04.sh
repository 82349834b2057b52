#!/bin/bash
# Round 4, call g04: BN-backward reduction in the dgrad epilogues at the default batch (1280).
#  A/B (interleaved x2): default vs BN_EPILOGUE=stream (only the persistent streaming 1x1 data gradients
#  carry the reduction) vs BN_EPILOGUE=1 (every dgrad); then one rocprofv3 kernel trace per mode.
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
done
