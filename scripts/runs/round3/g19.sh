#!/bin/bash
# Round 3, call 19: late-joined weight gradients, "auto" mode (3x3 + 1x1 above an arithmetic-intensity
# threshold) vs 3x3 only vs off; interleaved, 3 rounds.
set -o pipefail
O=gpurun_out/g19; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad_defer.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2 3; do
  for v in 0:0 3x3:0 auto:100 auto:200 auto:400; do
    d=${v%%:*}; a=${v##*:}
    DLA_WGRAD_DEFER=$d DLA_WGRAD_DEFER_MIN_AI=$a timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${d}_${a}_$i.log 2>&1 || { tail -30 $O/bench_${d}_${a}_$i.log; exit 1; }
    echo "defer=$d min_ai=$a $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${d}_${a}_$i.log)" | tee -a $O/ab.txt
  done
done
