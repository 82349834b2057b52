#!/bin/bash
# A/B of the side-stream weight-gradient overlap threshold (ops/conv.py WGRAD_OVERLAP_MAX_ROWS) on the
# ResNet-50 bench, one GPU. Writes gpurun_out/wgo_<rows>.log.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for rows in 0 50176 200704 802816; do
  timeout -k 10 300 python $R/bench.py --steps 20 --warmup 8 --wgrad_overlap_rows $rows > $R/gpurun_out/wgo_$rows.log 2>&1 || exit $?
done
