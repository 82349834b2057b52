#!/bin/bash
# Headline scaling sweep: bench.py at 1, 2, 4, 8 GPUs (weak scaling, per-GPU batch fixed).
#   scripts/scaling_sweep.sh [bench flags...]   -> one JSON line per N in results/scaling.jsonl
set -uo pipefail
cd "$(dirname "$0")/.."
mkdir -p results
export HSA_ENABLE_IPC_MODE_LEGACY=0
for N in 1 2 4 8; do
  if [ "$N" -eq 1 ]; then
    timeout -k 10 1200 python bench.py --gpus 1 "$@" | tail -1 >> results/scaling.jsonl || break
  else
    timeout -k 10 1200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29600 + N)) bench.py --gpus $N "$@" | tail -1 >> results/scaling.jsonl || break
  fi
done
cat results/scaling.jsonl
