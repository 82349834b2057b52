#!/bin/bash
# Round 3, call 13: (1) streaming-GEMM tests under the default policy; (2) the GoogLeNet bs128 fp32 parity
# anchor through the CLI with MIOpen's kernel cache warm (a first fp32 run on a fresh box compiles MIOpen's
# backward kernels inside the measured phase's first batch, ~40 s: g08b); then fp32 and bf16 measured;
# (3) bench.py x2 and a kernel-trace profile of the default step.
set -o pipefail
O=gpurun_out/g13; mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_stream.py tests/test_gpu_halo_wgrad.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 python -u scripts/bench_halo_wgrad.py > $O/halo_wgrad.log 2>&1 || { tail -20 $O/halo_wgrad.log; exit 1; }
cat $O/halo_wgrad.log
timeout -k 10 400 python -u scripts/bench_gemm_stream.py --out $O/layers.jsonl > $O/layers.log 2>&1 || { tail -30 $O/layers.log; exit 1; }
grep fork $O/layers.jsonl
CLI="python -u -m distributed_learning_amd.main 1 0 1 1 127.0.0.1 lo"
timeout -k 10 240 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 3 --precision fp32 --results_root $O/res_fp32_cold --job_id cold > $O/cli_g_fp32_cold.log 2>&1 || { tail -30 $O/cli_g_fp32_cold.log; exit 1; }
timeout -k 10 240 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 30 --precision fp32 --results_root $O/res_fp32 --job_id gfp32 > $O/cli_g_fp32.log 2>&1 || { tail -30 $O/cli_g_fp32.log; exit 1; }
timeout -k 10 240 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 30 --results_root $O/res_bf16 --job_id gbf16 > $O/cli_g_bf16.log 2>&1 || { tail -30 $O/cli_g_bf16.log; exit 1; }
python scripts/cli_vs_bench.py --cli $O/res_fp32_cold/experiment_single_1_cold --cli $O/res_fp32/experiment_single_1_gfp32 --cli $O/res_bf16/experiment_single_1_gbf16 > $O/googlenet_cli.json
grep -h '"img_s"' $O/googlenet_cli.json
for i in 1 2; do
  for cfg in "DLA_HALO_WGRAD=1 DLA_GEMM_STREAM=1" "DLA_HALO_WGRAD=0 DLA_GEMM_STREAM=1" "DLA_HALO_WGRAD=1 DLA_GEMM_STREAM=0"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${tag}_$i.log 2>&1 || { tail -30 $O/bench_${tag}_$i.log; exit 1; }
    echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${tag}_$i.log)" | tee -a $O/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g13prof -o prof -- python3 $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1 || { tail -30 $R/$O/prof.log; exit 1; }
cd $R
T=$(find /tmp/g13prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 20 --out $O/ksum > /dev/null
S=$(find /tmp/g13prof -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats.csv
head -22 $O/ksum.md
