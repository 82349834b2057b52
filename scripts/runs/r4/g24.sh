#!/bin/bash
# Round 4, call g24: short final-tree check (the pool was too busy for g23's full suite): the one-pass gradient
# kernel tests, model parity, smoke() and the driver's bench command twice
set -o pipefail
O=gpurun_out/g24
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_dual.py tests/test_gpu_model_parity.py -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep metric $O/bench.log | cut -c1-400
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 1; }
grep metric $O/bench2.log | cut -c1-400
