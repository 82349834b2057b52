#!/bin/bash
# Round 6, call g01: stall attribution of the stage-3/4 128x128 1x1 GEMMs (verdict r5 item 1a) -- plain timings,
# 4 counter passes per shape (each its own run), kernel resource usage from a kernel trace; then the driver's bench
# command once for the box's clock class.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r6/g01
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" $O/avail.txt && printf '%s ' "$c"; done; }
P1=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS)
P2=$(have SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS)
P3=$(have TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum)
P4=$(have SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAIT_INST_LDS)
echo "P1=$P1"; echo "P2=$P2"; echo "P3=$P3"; echo "P4=$P4"
SH=("250880 256 1024 fwd" "250880 256 1024 dgrad_add" "62720 512 2048 fwd" "62720 512 2048 dgrad_add" "1003520 512 128 dgrad_add" "1003520 256 512 fwd")
for s in "${SH[@]}"; do
  timeout -k 10 120 python3 $R/scripts/gemm_stall.py $s 40 >> $O/timing.txt 2>&1 || { tail $O/timing.txt; exit 1; }
done
cat $O/timing.txt
i=0
for s in "${SH[@]}"; do
  i=$((i+1))
  for p in 1 2 3 4; do
    eval C=\$P$p
    [ -z "$C" ] && continue
    timeout -s KILL 90 rocprofv3 --pmc $C GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc_s${i}_p$p -o p -- python3 $R/scripts/gemm_stall.py $s 12 > $O/pmc_s${i}_p$p.log 2>&1 || { tail -5 $O/pmc_s${i}_p$p.log; exit 1; }
    f=$(find /tmp/pmc_s${i}_p$p -name '*counter_collection.csv' | head -1)
    cp "$f" $O/s${i}_p$p.csv
  done
  echo "shape $i ($s) counters done"
done
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt1 -o k -- python3 $R/scripts/gemm_stall.py 250880 256 1024 fwd 6 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
cp $(find /tmp/kt1 -name '*kernel_trace.csv' | head -1) $O/kt_fwd.csv
cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.jsonl').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['telemetry']['before_timed'])"
