#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_tiles_r2.py > gpurun_out/r2d_tiles.log 2>&1; echo "tiles rc=$?"; cat gpurun_out/r2d_tiles.log | tail -12
timeout -k 10 300 python bench.py --model googlenet --batch 128 --steps 20 --warmup 5 --graph on > gpurun_out/r2d_gnet_graph.log 2>&1; echo "gnet graph rc=$?"; grep metric gpurun_out/r2d_gnet_graph.log || tail -20 gpurun_out/r2d_gnet_graph.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2d_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r2d_smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model_parity.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r2d_parity.log 2>&1; echo "parity rc=$?"; grep -E "passed|failed|native:|fp32  :" gpurun_out/r2d_parity.log
