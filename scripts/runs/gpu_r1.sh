set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export MIOPEN_USER_DB_PATH=$R/miopen_db
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_bench_prof.sh r1s2
