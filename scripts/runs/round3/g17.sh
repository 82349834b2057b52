#!/bin/bash
# Round 3, call 17: BN pass row-traversal orders (MALL reuse between consecutive passes): numerics of every
# order, then an interleaved end-to-end A/B of DLA_BN_ORDER bit sets, 2 rounds.
set -o pipefail
O=gpurun_out/g17; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn_act.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for v in 0 1 3 13 2 8; do
    DLA_BN_ORDER=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "order=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
