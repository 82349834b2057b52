#!/bin/bash
# Round 3, call 41: late weight gradients skipped inside HIP-graph capture: GoogLeNet bs128 --graph on,
# defer 0 vs 3x3 (2 rounds); graph tests.
set -o pipefail
O=gpurun_out/g41; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_wgrad_defer.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for d in 0 3x3; do
    DLA_WGRAD_DEFER=$d timeout -k 10 300 python3 bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > $O/g_${d}_$i.log 2>&1 || { tail -20 $O/g_${d}_$i.log; exit 1; }
    echo "gnet128g defer=$d $(grep -o '"value": [0-9.]*' $O/g_${d}_$i.log | head -1)" | tee -a $O/ab.txt
  done
done
