#!/bin/bash
# PMC passes (one counter set per run) on the stage-1 3x3 conv kernels (implicit GEMM, halo v1 / v2)
# and the short-K 1x1 forward GEMM with the BN-statistics epilogue
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out/r5k; cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
run() {  # tag halo halo_v args...
  tag=$1; h=$2; v=$3; shift 3
  for p in 1 2; do
    if [ $p = 1 ]; then C=$P1; else C=$P2; fi
    DLA_HALO=$h DLA_HALO_V=$v timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d /tmp/pm_${tag}_$p -o p -- python3 $R/scripts/conv_one.py "$@" 20 > $R/gpurun_out/r5k/$tag.log 2>&1 || return 1
  done
  find /tmp/pm_${tag}_1 /tmp/pm_${tag}_2 -name '*counter_collection.csv' > /tmp/list_$tag
  python3 $R/scripts/pmc_table.py $(cat /tmp/list_$tag) > $R/gpurun_out/r5k/$tag.md
}
run fwd_igemm 0 1 fwd 64 56 64 1 || exit 1
run fwd_halo1 2 1 fwd 64 56 64 1 || exit 1
run fwd_halo2 2 2 fwd 64 56 64 1 || exit 1
run dgrad_halo1 1 1 dgrad 64 56 64 1 || exit 1
run gemm_k64 1 1 gemm 802816 64 256 1 || exit 1
head -50 $R/gpurun_out/r5k/*.md
