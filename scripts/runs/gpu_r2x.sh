#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for v in 2 -1 2 -1 2 -1; do
  if [ "$v" = "-1" ]; then unset DLA_CONV_PIPE; else export DLA_CONV_PIPE=$v; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r2x_bench.log 2>&1 && echo "conv_pipe=$v $(grep -o '"value": [0-9.]*' gpurun_out/r2x_bench.log | head -1)"
done
