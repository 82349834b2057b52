#!/bin/bash
# GoogLeNet: BN-backward reduction in the consumer dgrad epilogue (DLA_BN_EPILOGUE) A/B
set -o pipefail
mkdir -p gpurun_out
for v in 1 0 1 0; do
  DLA_BN_EPILOGUE=$v timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > gpurun_out/r4b_g.log 2>&1 && echo "gnet epi=$v $(grep -o '"value": [0-9.]*' gpurun_out/r4b_g.log | head -1)"
done
for v in 1 0; do
  DLA_BN_EPILOGUE=$v timeout -k 10 300 python bench.py --model googlenet --batch 512 --steps 20 --warmup 5 > gpurun_out/r4b_g5.log 2>&1 && echo "gnet512 epi=$v $(grep -o '"value": [0-9.]*' gpurun_out/r4b_g5.log | head -1)"
done
