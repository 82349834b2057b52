#!/bin/bash
# Round 5, call g57: 512x128 tile for the stage-2 stride-2 3x3 data gradient: conv GPU tests, per-kernel A/B
set -o pipefail
O=gpurun_out/r5/g57
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_tile_policy.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  DLA_TILE512=0 timeout -k 10 120 python -u scripts/probe_s2dgrad.py >> $O/probe.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  timeout -k 10 120 python -u scripts/probe_s2dgrad.py >> $O/probe.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
cat $O/probe.jsonl
