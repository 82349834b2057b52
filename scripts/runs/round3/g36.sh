#!/bin/bash
# Round 3, call 36: late 3x3 weight gradients on the 128x128 4-wave tiles (blocks leave room for the
# compute stream's BN passes) vs the 256x256 8-wave tiles; bitwise-defer tests; 3 interleaved rounds.
set -o pipefail
O=gpurun_out/g36; mkdir -p $O
DLA_WGRAD_DEFER_TILE=narrow timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_defer.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2 3; do
  for v in wide narrow; do
    DLA_WGRAD_DEFER_TILE=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
