#!/bin/bash
# model parity vs fp32 torch, smoke, GoogLeNet bench + kernel profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_model_parity.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r2c_parity.log 2>&1
echo "parity rc=$?"; grep -E "PASS|FAIL|Error|assert|native:|fp32  :|largest" gpurun_out/r2c_parity.log | head -30
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c_smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/r2c_smoke.log
timeout -k 10 300 python bench.py --model googlenet --batch 128 --steps 20 --warmup 5 > gpurun_out/r2c_googlenet.log 2>&1; echo "gnet rc=$?"; grep metric gpurun_out/r2c_googlenet.log || tail -20 gpurun_out/r2c_googlenet.log
bash scripts/gpu_bench_prof.sh r2c_gnet --model googlenet --batch 128 || echo "prof failed"
head -60 gpurun_out/ksum_r2c_gnet.md
