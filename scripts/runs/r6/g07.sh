#!/bin/bash
# Round 6, call g07: fp32 convs with rectangular tiles (least padded work) -- tests, per-layer vs MIOpen, counters of
# two large 3x3 layers (forward and weight gradient), fp32 GoogLeNet line
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r6/g07
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_f32.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
timeout -k 10 500 python -u scripts/bench_conv_f32.py --out $O/layers.jsonl > $O/layers.log 2>&1 || { tail -20 $O/layers.log; exit 1; }
tail -1 $O/layers.log
timeout -k 10 300 python bench.py --model googlenet --precision fp32 --batch 128 --steps 20 --warmup 5 > $O/gnet_fp32.jsonl 2> $O/gnet.err || { tail $O/gnet.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/gnet_fp32.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['conv1x1'])"
cd /tmp && export TMPDIR=/tmp
i=0
for s in "128 128 14 256 3 1 fwd" "128 64 56 192 3 1 fwd" "128 128 14 256 3 1 wgrad"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d /tmp/pf_$i -o p -- python3 $R/scripts/conv_f32_one.py $s 10 > $O/pmc_$i.log 2>&1 || { tail -5 $O/pmc_$i.log; exit 1; }
  cp $(find /tmp/pf_$i -name '*counter_collection.csv' | head -1) $O/pmc_$i.csv
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE \
    --output-format csv -d /tmp/pg_$i -o p -- python3 $R/scripts/conv_f32_one.py $s 10 > $O/pmcb_$i.log 2>&1 || { tail -5 $O/pmcb_$i.log; exit 1; }
  cp $(find /tmp/pg_$i -name '*counter_collection.csv' | head -1) $O/pmcb_$i.csv
  python3 $R/scripts/pmc_table.py $O/pmc_$i.csv $O/pmcb_$i.csv --match gemm_f32 > $O/counters_$i.txt
done
cat $O/counters_1.txt
