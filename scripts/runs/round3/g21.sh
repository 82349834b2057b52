#!/bin/bash
# Round 3, call 21: downsample shortcut conv on a branch stream (DLA_BRANCH_STREAM): bitwise tests, then an
# interleaved end-to-end A/B, 3 rounds.
set -o pipefail
O=gpurun_out/g21; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_branch_stream.py tests/test_gpu_wgrad_defer.py tests/test_gpu_uninit.py tests/test_gpu_gemm_stream.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2 3; do
  for v in 0 1; do
    DLA_BRANCH_STREAM=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "branch=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
