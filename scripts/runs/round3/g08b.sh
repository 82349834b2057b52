#!/bin/bash
# Round 3, call 8b: the rest of g08 after its GoogLeNet fp32 CLI run stalled (fp32 ran channels_last with
# MIOpen exhaustive find; now NCHW + immediate mode): GoogLeNet bs128 CLI fp32 + bf16 parity anchor, ring /
# channel timing on virtual ranks, gradient-hook host cost at ResNet-152 / GoogLeNet tensor counts.
set -o pipefail
O=gpurun_out/g08b; mkdir -p $O
CLI="python -u -m distributed_learning_amd.main 1 0 1 1 127.0.0.1 lo"
timeout -k 10 240 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 30 --precision fp32 --results_root $O/res_fp32 --job_id gfp32 > $O/cli_g_fp32.log 2>&1 || { tail -30 $O/cli_g_fp32.log; exit 1; }
timeout -k 10 240 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 30 --results_root $O/res_bf16 --job_id gbf16 > $O/cli_g_bf16.log 2>&1 || { tail -30 $O/cli_g_bf16.log; exit 1; }
python scripts/cli_vs_bench.py --cli $O/res_fp32/experiment_single_1_gfp32 --cli $O/res_bf16/experiment_single_1_gbf16 > $O/googlenet_cli.json
grep -h '"img_s"' $O/googlenet_cli.json
timeout -k 10 200 python -u scripts/vrank_ring_timing.py --out $O/vrank_eager.jsonl > $O/vrank_eager.log 2>&1 || { tail -20 $O/vrank_eager.log; exit 1; }
timeout -k 10 200 python -u scripts/vrank_ring_timing.py --graph --out $O/vrank_graph.jsonl > $O/vrank_graph.log 2>&1 || { tail -20 $O/vrank_graph.log; exit 1; }
for i in 1 2; do
  for fc in 1 0; do
    DLA_HOOK_TIMING=1 timeout -k 10 200 python3 bench.py --model resnet152 --batch 256 --steps 20 --warmup 5 --force_comm $fc > $O/r152_fc${fc}_$i.log 2>&1 || { tail -20 $O/r152_fc${fc}_$i.log; exit 1; }
    DLA_HOOK_TIMING=1 timeout -k 10 200 python3 bench.py --model googlenet --batch 128 --steps 30 --warmup 5 --force_comm $fc > $O/gn_fc${fc}_$i.log 2>&1 || { tail -20 $O/gn_fc${fc}_$i.log; exit 1; }
    for m in r152 gn; do echo "$m fc=$fc $(grep -o '"ms_per_step": [0-9.]*\|"hook_host_ms_per_step": [0-9.]*\|"allreduce_ms_per_step": [0-9.]*\|"hook_calls_per_step": [0-9.]*' $O/${m}_fc${fc}_$i.log | tr '\n' ' ')" | tee -a $O/hooks_ab.txt; done
  done
done
bash scripts/runs/round3/g10.sh
