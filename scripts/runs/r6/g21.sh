#!/bin/bash
# Round 6, call g21: the deferred block-final apply on the bench's other paths -- HIP-graph replay, autocast, the
# forced multi-rank data path (fusion off, strict), and two real ranks on one GPU (IPC transport)
set -o pipefail
O=gpurun_out/r6/g21
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 "$@" > $O/$n.jsonl 2> $O/$n.err || { echo "$n failed"; tail $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.jsonl').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['config'].get('parallelism'), d.get('kernels'))"
}
run r50_bs256_graph --batch 256 --graph on
DLA_DEFER_APPLY=0 run r50_bs256_graph_nodefer --batch 256 --graph on
run r50_bs256_autocast --batch 256 --precision autocast
DLA_LAUNCH_GROUPS=0 run r50_bs256_fusion_off --batch 256 --force_comm 1 --bucket_mb 0
run r50_dp2_same_device --gpus 2 --same_device 1 --batch 256
