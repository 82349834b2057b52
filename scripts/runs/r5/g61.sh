#!/bin/bash
# Round 5, call g61: N>1 bench path on the final tree (two ranks, one GPU, IPC transport) and the multi-process GPU tests
# (autotune probe engines, measured bucket cap, MAX-over-ranks JSON)
set -o pipefail
O=gpurun_out/r5/g61
mkdir -p $O
export DLA_COMM_TIMEOUT_S=60
timeout -k 10 400 python bench.py --gpus 2 --same_device 1 --batch 64 --steps 4 --warmup 2 > $O/bench2.log 2>&1 || { tail -30 $O/bench2.log; exit 1; }
grep metric $O/bench2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d['config'], json.dumps(d.get('allreduce_table',{}).get('excluded')), d['allreduce_table'].get('cap_backward_ms'), d['allreduce_table'].get('probe_engines'))"
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiproc.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/multiproc.log 2>&1 || { echo "multiproc tests failed"; tail -30 $O/multiproc.log; exit 1; }
tail -1 $O/multiproc.log
