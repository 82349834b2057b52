#!/bin/bash
# Round 3, call 32: late weight gradients on a CU-masked side stream (1/n of every XCD's CUs kept free for
# the compute stream): n = 0 (unrestricted), 8, 4; interleaved, 3 rounds; bitwise tests with n = 4.
set -o pipefail
O=gpurun_out/g32; mkdir -p $O
DLA_SIDE_CU_RESERVE=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_defer.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2 3; do
  for v in 0 8 4; do
    DLA_SIDE_CU_RESERVE=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "reserve=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
