#!/bin/bash
# Round 3, call 39: halo-tiled stem forward: stem tests, micro-bench, end-to-end A/B (3 rounds).
set -o pipefail
O=gpurun_out/g39; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_pool.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 python3 scripts/bench_stem.py > $O/stem.log 2>&1 || { tail -20 $O/stem.log; exit 1; }
grep '^{' $O/stem.log
for i in 1 2 3; do
  for v in 1 0; do
    DLA_STEM_HALO=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "stem_halo=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
