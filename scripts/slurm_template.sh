#!/bin/bash
# SLURM template (reference: submit.sh). One task per node, torchrun spawns one process per GPU;
# multi-node rendezvous over the first node of the allocation.
#SBATCH -J dla
#SBATCH --nodes=2
#SBATCH --ntasks-per-node=1
#SBATCH --gpus-per-node=8
#SBATCH --time=00:30:00
#SBATCH --no-requeue
set -euo pipefail
MASTER=$(scontrol show hostnames "$SLURM_JOB_NODELIST" | head -n1)
export HSA_ENABLE_IPC_MODE_LEGACY=0
srun python -m torch.distributed.run --nnodes="$SLURM_NNODES" --nproc-per-node=8 \
    --rdzv-backend=c10d --rdzv-endpoint="$MASTER:29501" --rdzv-id="$SLURM_JOB_ID" \
    -m distributed_learning_amd.main --experiment "${EXPERIMENT:-experiment2}" --job_id "$SLURM_JOB_ID" \
    --model "${MODEL:-resnet50}" --random_input 1 --limit_batches "${BATCHES:-30}" --local_size 8
