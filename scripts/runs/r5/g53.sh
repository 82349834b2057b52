#!/bin/bash
# Round 5, call g53: the round-end sequence on the final tree (after g48 BN order, g50 wgrad loop) -- full GPU suite, smoke, driver bench command x2
set -o pipefail
O=gpurun_out/r5/g53
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/full_gpu.log 2>&1 || { echo "GPU suite failed"; grep -E "Error|assert|FAIL|failed" $O/full_gpu.log | head -20; tail -30 $O/full_gpu.log; exit 1; }
tail -2 $O/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
done
grep metric $O/bench.jsonl | cut -c1-260
