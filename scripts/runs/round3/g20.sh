#!/bin/bash
# Round 3, call 20: full GPU suite + smoke + driver bench with the late-joined 3x3 weight gradients on by
# default; GoogLeNet bs128 under the HIP graph (side-stream fork/join inside capture).
set -o pipefail
O=gpurun_out/g20; mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
timeout -k 10 300 python3 bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > $O/gnet_graph.log 2>&1 || { tail -30 $O/gnet_graph.log; exit 1; }
grep -o '"value": [0-9.]*' $O/gnet_graph.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "Error|assert|FAIL|failed" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
