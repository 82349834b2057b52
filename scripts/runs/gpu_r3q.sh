#!/bin/bash
# max-pool microbenchmark at GoogLeNet branch-4 shapes + one PMC pass on the 14x14x480 forward
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
timeout -k 10 120 python $R/scripts/pool_probe.py > $R/gpurun_out/r3q_pool.jsonl 2> $R/gpurun_out/r3q_pool.err || { tail -5 $R/gpurun_out/r3q_pool.err; exit 1; }
cat $R/gpurun_out/r3q_pool.jsonl
