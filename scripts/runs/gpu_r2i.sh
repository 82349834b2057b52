#!/bin/bash
# A/B: 16x16x32 vs 32x32x16 MFMA builds (same box): correctness, per-layer conv time, bench
set -o pipefail
mkdir -p gpurun_out
V=distributed_learning_amd/_variants/_C_mfma32.so
DLA_EXT_SO=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv3x3.py tests/test_gpu_conv.py tests/test_gpu_stem.py tests/test_gpu_bn_epilogue.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2i_tests32.log 2>&1 || { echo "mfma32 tests failed"; tail -40 gpurun_out/r2i_tests32.log; exit 1; }
tail -1 gpurun_out/r2i_tests32.log
for v in 16 32 16 32; do
  if [ $v = 32 ]; then export DLA_EXT_SO=$V; else unset DLA_EXT_SO; fi
  timeout -k 10 300 python -u scripts/bench_layers.py --pipe 6 --out gpurun_out/layers_r2i_m$v.jsonl > gpurun_out/layers_r2i_m$v.log 2>&1 || { echo "layers $v failed"; tail gpurun_out/layers_r2i_m$v.log; exit 1; }
  echo "mfma$v"; tail -7 gpurun_out/layers_r2i_m$v.log
done
unset DLA_EXT_SO
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r2i_bench16.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/r2i_bench16.log
DLA_EXT_SO=$V timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r2i_bench32.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/r2i_bench32.log
