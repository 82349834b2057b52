#!/bin/bash
# Round 3, call 43: MFMA utilisation table again (kernel-name fix for the anonymous-namespace kernels).
set -o pipefail
timeout -k 10 360 bash scripts/gpu_pmc_mfma.sh || exit 1
head -40 gpurun_out/mfma_util.md
