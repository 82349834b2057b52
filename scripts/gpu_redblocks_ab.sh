#!/bin/bash
# BN reduction-pass block target A/B (DLA_BN_RED_BLOCKS): BN tests at 4096, then bench per target
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export MIOPEN_USER_DB_PATH=$R/miopen_db
DLA_BN_RED_BLOCKS=4096 timeout -k 10 300 python -u -m pytest tests/test_gpu_bn_act.py tests/test_gpu_pool.py tests/test_gpu_stem.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_redblocks.log 2>&1 || exit $?
for b in 1024 2048 4096; do
  DLA_BN_RED_BLOCKS=$b timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/bench_red$b.log 2>&1 || exit $?
done
