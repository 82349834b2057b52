export MIOPEN_USER_DB_PATH=$PWD/miopen_db
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r1s15.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_r1s15.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/bench_ab_epi0.log 2>&1 || exit $?
DLA_BN_EPILOGUE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/bench_ab_epi1.log 2>&1 || exit $?
exit $rc
