#!/bin/bash
# PMC: 3x3 wgrad vs fwd at the stage-2 shape (Cin = Cout = 128, 28x28, batch 256)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out/r2q; cd /tmp && export TMPDIR=/tmp
for op in fwd wgrad; do
  tag=$op
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k_$tag -o p -- python3 $R/scripts/conv_one.py $op 128 28 128 1 30 > $R/gpurun_out/r2q/$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d /tmp/a_$tag -o p -- python3 $R/scripts/conv_one.py $op 128 28 128 1 30 >> $R/gpurun_out/r2q/$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d /tmp/b_$tag -o p -- python3 $R/scripts/conv_one.py $op 128 28 128 1 30 >> $R/gpurun_out/r2q/$tag.log 2>&1 || exit 1
  mkdir -p $R/gpurun_out/r2q/$tag
  for d in k a b; do find /tmp/${d}_$tag \( -name '*counter_collection.csv' -o -name '*kernel_stats.csv' \) -exec cp {} $R/gpurun_out/r2q/$tag/${d}_counters_or_stats.csv \; ; done
done
python3 $R/scripts/pmc_table.py $R/gpurun_out/r2q/*/a_counters_or_stats.csv $R/gpurun_out/r2q/*/b_counters_or_stats.csv > $R/gpurun_out/r2q/table.txt 2>&1; cat $R/gpurun_out/r2q/table.txt | head -80
