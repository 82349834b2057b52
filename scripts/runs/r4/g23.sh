#!/bin/bash
# Round 4, call g23: round-end tier on the final tree (4-stage Cout-512 ring) -- full GPU suite, then smoke() and the
# driver's bench command
set -o pipefail
O=gpurun_out/g23
mkdir -p $O
timeout -k 10 960 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/full_gpu.log 2>&1 || { tail -30 $O/full_gpu.log; exit 1; }
tail -2 $O/full_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep metric $O/bench.log | cut -c1-400
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 1; }
grep metric $O/bench2.log | cut -c1-400
