#!/bin/bash
# Round 3, call 33: split-K block target of the late 3x3 weight gradients only (shorter blocks free CUs for
# the compute stream's short kernels sooner): default (512), 1024, 2048; 3 rounds, interleaved.
set -o pipefail
O=gpurun_out/g33; mkdir -p $O
for i in 1 2 3; do
  for v in 0 1024 2048; do
    DLA_WGRAD_DEFER_SPLITK_BLOCKS=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "defer_splitk_blocks=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
