#!/bin/bash
# Round-2 first GPU pass: virtual-rank engine tests, the full GPU suite, the bench, the 2-rank probe.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine_vranks.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r2a_vranks.log 2>&1 || { echo "vranks failed rc=$?"; tail -40 gpurun_out/r2a_vranks.log; exit 1; }
tail -3 gpurun_out/r2a_vranks.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/r2a_gpu_tests.log 2>&1 || { echo "gpu suite failed rc=$?"; tail -40 gpurun_out/r2a_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r2a_gpu_tests.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/r2a_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r2a_bench.log; exit 1; }
grep metric gpurun_out/r2a_bench.log
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  scripts/multirank_probe.py > gpurun_out/r2a_probe.log 2>&1
echo "probe rc=$?"
tail -15 gpurun_out/r2a_probe.log
