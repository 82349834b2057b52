#!/bin/bash
# bench + steady-state kernel profile on one GPU (run from the repo root on the GPU box)
#   bash scripts/gpu_bench_prof.sh TAG [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}
shift
mkdir -p $R/gpurun_out
export MIOPEN_USER_DB_PATH=${MIOPEN_USER_DB_PATH:-$R/miopen_db}
timeout -k 10 900 python $R/bench.py --steps 20 --warmup 10 "$@" > $R/gpurun_out/bench_$TAG.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_$TAG -o prof -- python3 $R/bench.py --steps 8 --warmup 4 "$@" > $R/gpurun_out/prof_$TAG.log 2>&1 || exit $?
T=$(find /tmp/prof_$TAG -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/kernel_summary.py "$T" --steps 8 --out $R/gpurun_out/ksum_$TAG > /dev/null
mkdir -p $R/gpurun_out/miopen_db && cp -r $MIOPEN_USER_DB_PATH/. $R/gpurun_out/miopen_db/ 2>/dev/null
exit 0
