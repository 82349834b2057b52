#!/bin/bash
# Round 5, call g01: baseline of the round-4 tree on a fresh box -- the two-process IPC check run directly
# (its full per-rank output kept), the multi-process GPU tests, and the driver's bench command
set -o pipefail
O=gpurun_out/r5/g01
mkdir -p $O
export DLA_COMM_TIMEOUT_S=60
timeout -k 10 240 python -u scripts/ipc_engine_check.py --ranks 2 --same_device 1 --timeout 200 \
  > $O/ipc_check.out 2> $O/ipc_check.err; echo "ipc_check rc=$?" | tee $O/ipc_check.rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py -x -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/multiproc.log 2>&1; echo "multiproc rc=$?" | tee -a $O/ipc_check.rc
tail -5 $O/multiproc.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep metric $O/bench.log | cut -c1-600
