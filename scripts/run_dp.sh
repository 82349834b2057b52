#!/bin/bash
# Launch an experiment on N GPUs of one node, one process per GPU (RCCL over xGMI).
# Replaces the reference's mpirun/SLURM launchers (submit.sh, submits/submit2x*.sh).
#   scripts/run_dp.sh N EXPERIMENT [extra main.py flags...]
# e.g. scripts/run_dp.sh 8 experiment2 --model resnet50 --random_input 1 --limit_batches 30
set -euo pipefail
N=${1:-8}; EXP=${2:-experiment2}; shift 2 || true
PORT=${MASTER_PORT:-29501}
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$(dirname "$0")/.."
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port "$PORT" -m distributed_learning_amd.main --experiment "$EXP" --job_id "${JOB_ID:-local}" "$@"
