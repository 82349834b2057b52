#!/bin/bash
# Round 5, call g10: the fp32 GoogLeNet step -- native fp32 and stock fp32 both judged against a float64 run
set -o pipefail
O=gpurun_out/r5/g10
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp32_path.py -x -v -s --timeout 360 --timeout-method thread \
  -p no:cacheprovider > $O/test.log 2>&1; rc=$?
grep -E "vs fp64|PASSED|FAILED|Error" $O/test.log | head -20
exit $rc
