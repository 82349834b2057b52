#!/bin/bash
# One GPU session: tests, GEMM micro-bench, bench variants, steady-state profile of the best one.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export MIOPEN_USER_DB_PATH=$R/miopen_db
timeout -k 10 600 python -m pytest tests/test_gpu_gemm.py tests/test_gpu_bn_act.py tests/test_gpu_kernels.py -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1 || exit $?
for cfg in "--kernels native --precision bf16" "--kernels native --precision bf16 --conv native"; do
  tag=$(echo $cfg | tr -d ' -' )
  timeout -k 10 600 python bench.py $cfg > gpurun_out/bench_$tag.log 2>&1 || exit $?
done
bash scripts/gpu_bench_prof.sh nconv --kernels native --precision bf16 --conv native
