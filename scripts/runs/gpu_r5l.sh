#!/bin/bash
# halo v1 with one base address per (tap, k-half) + base select for padding taps: tests, per-layer
# A/B (off / v1 fwd+dgrad), counter pass, whole-step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out/r5l
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5l/conv_tests.log 2>&1 || { tail -40 gpurun_out/r5l/conv_tests.log; exit 1; }
tail -1 gpurun_out/r5l/conv_tests.log
for r in 1 2; do
  for h in 0 2; do
    DLA_HALO=$h timeout -k 10 240 python -u scripts/bench_layers.py --only fwd,dgrad --out gpurun_out/r5l/layers_h${h}_r$r.jsonl > gpurun_out/r5l/layers.log 2>&1 || { tail -20 gpurun_out/r5l/layers.log; exit 1; }
  done
done
grep -h s56_c2 gpurun_out/r5l/layers_h*_r*.jsonl | cut -c1-120
( cd /tmp && export TMPDIR=/tmp && DLA_HALO=2 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d /tmp/pm_l -o p -- python3 $R/scripts/conv_one.py fwd 64 56 64 1 20 > $R/gpurun_out/r5l/pmc.log 2>&1 ) || exit 1
python3 $R/scripts/pmc_table.py $(find /tmp/pm_l -name '*counter_collection.csv') > $R/gpurun_out/r5l/pmc_halo_fwd.md; cat $R/gpurun_out/r5l/pmc_halo_fwd.md
for i in 1 2; do
  for h in 2 1 0; do
    DLA_HALO=$h timeout -k 10 300 python bench.py > gpurun_out/r5l/bench_h${h}_${i}.log 2>&1 || { tail -20 gpurun_out/r5l/bench_h${h}_${i}.log; exit 1; }
    echo "halo=$h $(grep -o '"value": [0-9.]*' gpurun_out/r5l/bench_h${h}_${i}.log | head -1)" | tee -a gpurun_out/r5l/ab.txt
  done
done
