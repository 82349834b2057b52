#!/bin/bash
# BN-backward reduction in the dgrad GEMM epilogue: A/B on the current kernels
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 0 1 0 1; do
  DLA_BN_EPILOGUE=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r3b.log 2>&1 && echo "bn_epilogue=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3b.log | head -1)"
done
