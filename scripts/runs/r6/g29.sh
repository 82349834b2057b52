#!/bin/bash
# Round 6, call g29: stall attribution of the stage-1 halo 3x3 conv (64 -> 64 channels, 56x56, bs1280): forward and
# data gradient, 4 counter passes each (own runs), plain timing
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r6/g29
mkdir -p $O
export CONV_ONE_N=1280
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" $O/avail.txt && printf '%s ' "$c"; done; }
P1=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS)
P2=$(have SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS)
P3=$(have TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum)
P4=$(have SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAIT_INST_LDS)
echo "P1=$P1"; echo "P2=$P2"; echo "P3=$P3"; echo "P4=$P4"
SH=("fwd 64 56 64 1" "dgrad 64 56 64 1")
i=0
for s in "${SH[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$i -o k -- python3 $R/scripts/conv_one.py $s 20 > $O/kt_$i.log 2>&1 || { tail -5 $O/kt_$i.log; exit 1; }
  cp $(find /tmp/kt_$i -name '*kernel_stats.csv' | head -1) $O/s${i}_stats.csv
  for p in 1 2 3 4; do
    eval C=\$P$p
    [ -z "$C" ] && continue
    timeout -s KILL 90 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc_s${i}_p$p -o p -- python3 $R/scripts/conv_one.py $s 8 > $O/pmc_s${i}_p$p.log 2>&1 || { tail -5 $O/pmc_s${i}_p$p.log; exit 1; }
    f=$(find /tmp/pmc_s${i}_p$p -name '*counter_collection.csv' | head -1)
    cp "$f" $O/s${i}_p$p.csv
  done
  echo "shape $i ($s) counters done"
done
cd $R
for i in 1 2; do
  python3 scripts/pmc_table.py $O/s${i}_p*.csv --match halo > $O/counters_s$i.txt || exit 1
  cat $O/counters_s$i.txt
  grep -i halo $O/s${i}_stats.csv | cut -c1-200
done
