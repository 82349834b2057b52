#!/bin/bash
# Round 3, call 1: reproduce the driver's BENCH_r02 (90.05 ms/step) on a fresh box.
# (1) the driver's exact command first, before any other GPU work; (2) the same with 60 timed steps to see
#     whether steps speed up over time (ramp) or stay slow (box); (3) the exact command under rocprofv3
#     kernel-trace for a per-kernel diff against profiles/resnet50_bs1024_r5m_ksum.md.
set -o pipefail
O=gpurun_out/g01; mkdir -p $O
timeout -k 10 60 amd-smi static --limit --clock > $O/smi_static.txt 2>&1 || true
timeout -k 10 60 amd-smi metric --power --clock --temperature > $O/smi_metric_before.txt 2>&1 || true
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/exact.log 2>&1 || { tail -30 $O/exact.log; exit 1; }
grep '^{' $O/exact.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 60 --warmup 5 > $O/long.log 2>&1 || { tail -30 $O/long.log; exit 1; }
grep '^{' $O/long.log
R=$(pwd); export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g01prof -o prof -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
grep '^{' $O/prof.log
T=$(find /tmp/g01prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 20 --out $O/ksum > /dev/null
S=$(find /tmp/g01prof -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
timeout -k 10 60 amd-smi metric --power --clock --temperature > $O/smi_metric_after.txt 2>&1 || true
