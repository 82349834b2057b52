#!/bin/bash
# PMC wait-state breakdown of the 3x3 forward kernel variants (one counter pass per run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out/r2f; cd /tmp && export TMPDIR=/tmp
for v in "2 1" "4 1" "3 4"; do
  set -- $v; pipe=$1; tile=$2; tag=p${pipe}_t${tile}
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k_$tag -o p -- python3 $R/scripts/conv_one.py fwd 256 14 256 1 30 $pipe $tile > $R/gpurun_out/r2f/$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d /tmp/a_$tag -o p -- python3 $R/scripts/conv_one.py fwd 256 14 256 1 30 $pipe $tile >> $R/gpurun_out/r2f/$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d /tmp/b_$tag -o p -- python3 $R/scripts/conv_one.py fwd 256 14 256 1 30 $pipe $tile >> $R/gpurun_out/r2f/$tag.log 2>&1 || exit 1
  mkdir -p $R/gpurun_out/r2f/$tag
  for d in k a b; do find /tmp/${d}_$tag \( -name '*counter_collection.csv' -o -name '*kernel_stats.csv' \) -exec cp {} $R/gpurun_out/r2f/$tag/${d}_counters_or_stats.csv \; ; done
done
ls -R $R/gpurun_out/r2f | head -30
