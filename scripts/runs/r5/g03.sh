#!/bin/bash
# Round 5, call g03: g02 again after the backward calibration moved into the warmup steps (g02: the oracle test
# generations, barrier-timeout record), autotune probe engines, the BN hand-off guards, the one-pass kernels
# at the bench rows, smoke reaching the one-pass kernels, and the bench
set -o pipefail
O=gpurun_out/r5/g03
mkdir -p $O
export DLA_COMM_TIMEOUT_S=60
timeout -k 10 700 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_gemm_dual.py tests/test_gpu_bench_batch.py \
  -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|ipc check" $O/tests.log | tail -40
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 2 --same_device 1 --batch 64 --steps 4 --warmup 2 > $O/bench2.log 2>&1 || { tail -30 $O/bench2.log; exit 1; }
grep metric $O/bench2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['bucket_mb'], json.dumps(d.get('allreduce_table',{}).get('excluded')), d['allreduce_table'].get('cap_backward_ms'), d['allreduce_table'].get('probe_engines'))"
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep metric $O/bench.log | cut -c1-300
