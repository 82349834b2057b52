#!/bin/bash
# Round 3, call 37: stream-K 256x256 conv forward: tests, per-layer timing, end-to-end A/B (3 rounds).
set -o pipefail
O=gpurun_out/g37; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv3x3.py -x -q -k "streamk or fwd_dgrad_wgrad" --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 python3 scripts/bench_streamk.py > $O/layers.log 2>&1 || { tail -20 $O/layers.log; exit 1; }
grep '^{' $O/layers.log
for i in 1 2 3; do
  for v in 0 1; do
    DLA_STREAMK=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "streamk=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
