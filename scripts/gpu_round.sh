#!/bin/bash
# One GPU round: gpu tests, GEMM microbench, bench variants, kernel profile. Stops at the first
# crash / timeout (exit status >= 124); a plain test failure (rc 1) still runs the benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export MIOPEN_USER_DB_PATH=$R/miopen_db
TAG=${1:-round}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || exit $?
for cfg in "--kernels native --precision bf16" "--kernels native --precision bf16 --conv native"; do
  tag=$(echo $cfg | tr -d ' -' )
  timeout -k 10 600 python bench.py $cfg > gpurun_out/bench_$tag.log 2>&1 || exit $?
done
bash scripts/gpu_bench_prof.sh $TAG --kernels native --precision bf16
