#!/bin/bash
# MFMA utilisation of every kernel of the ResNet-50 training step (one counter pass, its own run).
#   bash scripts/gpu_pmc_mfma.sh [bench args...]  -> gpurun_out/mfma_util.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d /tmp/pmc_mfma -o p -- python3 $R/bench.py --steps 3 --warmup 2 "$@" \
  > $R/gpurun_out/pmc_mfma.log 2>&1 || exit $?
T=$(find /tmp/pmc_mfma -name '*counter_collection.csv' | head -1)
python3 $R/scripts/pmc_mfma.py "$T" --steps 2 --out $R/gpurun_out/mfma_util > /dev/null
