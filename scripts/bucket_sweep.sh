#!/bin/bash
# Fusion bucket-size sweep (BASELINE.json config "ResNet-152 large-batch ... bucket-size sweep"):
# bench.py over bucket sizes, one JSON line each -> gpurun_out/bucket_sweep_<model>.jsonl.
#   scripts/bucket_sweep.sh [N_GPUS] [MODEL] [BATCH] [extra bench flags...]
# N_GPUS > 1 launches torchrun (one rank per GPU, RCCL over xGMI); at N_GPUS = 1 add --force_comm 1
# to run the multi-rank gradient path (gather + RCCL all-reduce per bucket) on the single GPU.
set -uo pipefail
N=${1:-1}; MODEL=${2:-resnet152}; BATCH=${3:-256}; shift 3 || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 MIOPEN_USER_DB_PATH=${MIOPEN_USER_DB_PATH:-$R/miopen_db}
OUT=gpurun_out/bucket_sweep_${MODEL}_n${N}.jsonl
: > "$OUT"
for MB in 0 1 4 16 25 64 256; do
  if [ "$N" -eq 1 ]; then
    timeout -k 10 600 python bench.py --model "$MODEL" --batch "$BATCH" --bucket_mb $MB --steps 10 --warmup 5 "$@" \
      > gpurun_out/bucket_${MB}.log 2>&1 || exit $?
  else
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $((29700 + MB % 100)) bench.py --gpus "$N" --model "$MODEL" --batch "$BATCH" --bucket_mb $MB \
      --steps 10 --warmup 5 "$@" > gpurun_out/bucket_${MB}.log 2>&1 || exit $?
  fi
  tail -1 gpurun_out/bucket_${MB}.log >> "$OUT"
done
cat "$OUT"
