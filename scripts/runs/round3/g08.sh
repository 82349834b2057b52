#!/bin/bash
# Round 3, call 8: the full GPU suite + smoke (what the driver runs), CLI throughput vs bench.py
# (ResNet-50 bs1024), the GoogLeNet bs128 parity anchor through the CLI at fp32 and bf16, ring / channel
# timing on virtual ranks, and the gradient-hook host cost at ResNet-152 / GoogLeNet tensor counts.
set -o pipefail
O=gpurun_out/g08; mkdir -p $O
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/full_gpu.log 2>&1 || { echo "GPU suite failed"; grep -E "Error|assert|FAIL|failed" $O/full_gpu.log | head -20; tail -30 $O/full_gpu.log; exit 1; }
tail -2 $O/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
CLI="python -m distributed_learning_amd.main 1 0 1 1 127.0.0.1 lo"
timeout -k 10 300 $CLI resnet50 /none 1 --experiment experiment_single --batch_size 1024 --random_input 1 --limit_batches 30 --results_root $O/res --job_id r50 > $O/cli_r50.log 2>&1 || { tail -30 $O/cli_r50.log; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
timeout -k 10 300 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 30 --precision fp32 --results_root $O/res_fp32 --job_id gfp32 > $O/cli_g_fp32.log 2>&1 || { tail -30 $O/cli_g_fp32.log; exit 1; }
timeout -k 10 300 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 30 --results_root $O/res_bf16 --job_id gbf16 > $O/cli_g_bf16.log 2>&1 || { tail -30 $O/cli_g_bf16.log; exit 1; }
python scripts/cli_vs_bench.py --cli $O/res/experiment_single_1_r50 --bench $O/bench.log > $O/cli_vs_bench.json
python scripts/cli_vs_bench.py --cli $O/res_fp32/experiment_single_1_gfp32 --cli $O/res_bf16/experiment_single_1_gbf16 > $O/googlenet_cli.json
grep -h '"img_s"' $O/cli_vs_bench.json $O/googlenet_cli.json | head -10
timeout -k 10 200 python scripts/vrank_ring_timing.py --out $O/vrank_eager.jsonl > $O/vrank_eager.log 2>&1 || { tail -20 $O/vrank_eager.log; exit 1; }
timeout -k 10 200 python scripts/vrank_ring_timing.py --graph --out $O/vrank_graph.jsonl > $O/vrank_graph.log 2>&1 || { tail -20 $O/vrank_graph.log; exit 1; }
for i in 1 2; do
  for fc in 1 0; do
    DLA_HOOK_TIMING=1 timeout -k 10 300 python3 bench.py --model resnet152 --batch 256 --steps 20 --warmup 5 --force_comm $fc > $O/r152_fc${fc}_$i.log 2>&1 || { tail -20 $O/r152_fc${fc}_$i.log; exit 1; }
    DLA_HOOK_TIMING=1 timeout -k 10 300 python3 bench.py --model googlenet --batch 128 --steps 30 --warmup 5 --force_comm $fc > $O/gn_fc${fc}_$i.log 2>&1 || { tail -20 $O/gn_fc${fc}_$i.log; exit 1; }
    for m in r152 gn; do echo "$m fc=$fc $(grep -o '"ms_per_step": [0-9.]*\|"hook_host_ms_per_step": [0-9.]*\|"allreduce_ms_per_step": [0-9.]*\|"hook_calls_per_step": [0-9.]*' $O/${m}_fc${fc}_$i.log | tr '\n' ' ')" | tee -a $O/hooks_ab.txt; done
  done
done
