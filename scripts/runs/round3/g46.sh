#!/bin/bash
# Round 3, call 46: final-state validation (what the driver runs at round end): the driver's bench command,
# full GPU suite, smoke.
set -o pipefail
O=gpurun_out/g46; mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 && timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench2.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/bench.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "Error|assert|FAIL|failed" $O/gpu_tests.log | head -20; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
