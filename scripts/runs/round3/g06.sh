#!/bin/bash
# Round 3, call 6: virtual-y on the streaming kernels (vy_stream.hip; A/B + profile),
# teacher-forced parity against a bf16-storage fp32 reference, then the g03 items (teacher-forced parity, smoke, CLI tests, vrank timing, CLI vs bench, GoogLeNet fp32/bf16).
set -o pipefail
O=gpurun_out/g06; mkdir -p $O
R=$(pwd)
PT="python -u -m pytest -x -v -s --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_virtual_y.py > $O/pytest_vy.log 2>&1 || { tail -60 $O/pytest_vy.log; exit 1; }
tail -3 $O/pytest_vy.log
for i in 1 2; do
  for v in 1 0; do
    DLA_VIRTUAL_Y=$v timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_vy${v}_$i.log 2>&1 || { tail -30 $O/bench_vy${v}_$i.log; exit 1; }
    echo "vy=$v $(grep -o '"value": [0-9.]*' $O/bench_vy${v}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_vy${v}_$i.log)" | tee -a $O/ab.txt
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/g05prof6 -o prof -- python3 $R/bench.py --gpus 1 --steps 8 --warmup 4 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
T=$(find /tmp/g05prof6 -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 8 --out $O/ksum > /dev/null
head -16 $O/ksum.md
timeout -k 10 400 $PT tests/test_gpu_layer_parity.py > $O/pytest_parity.log 2>&1; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -60 $O/pytest_parity.log; exit 1; }
grep -E "segment|passed|failed" $O/pytest_parity.log | tail -50
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 $PT tests/test_gpu_cli.py > $O/pytest_cli.log 2>&1 || { tail -40 $O/pytest_cli.log; exit 1; }
tail -2 $O/pytest_cli.log
timeout -k 10 200 python scripts/vrank_ring_timing.py --out $O/vrank_eager.jsonl > $O/vrank_eager.log 2>&1 || { tail -20 $O/vrank_eager.log; exit 1; }
timeout -k 10 200 python scripts/vrank_ring_timing.py --graph --out $O/vrank_graph.jsonl > $O/vrank_graph.log 2>&1 || { tail -20 $O/vrank_graph.log; exit 1; }
CLI="python -m distributed_learning_amd.main 1 0 1 1 127.0.0.1 lo"
timeout -k 10 300 $CLI resnet50 /none 1 --experiment experiment_single --batch_size 1024 --random_input 1 --limit_batches 30 --results_root $O/res --job_id r50 > $O/cli_r50.log 2>&1 || { tail -30 $O/cli_r50.log; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
timeout -k 10 300 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 30 --precision fp32 --results_root $O/res_fp32 --job_id gfp32 > $O/cli_g_fp32.log 2>&1 || { tail -30 $O/cli_g_fp32.log; exit 1; }
timeout -k 10 300 $CLI imagenet /none 1 --experiment experiment_single --batch_size 128 --random_input 1 --limit_batches 30 --results_root $O/res_bf16 --job_id gbf16 > $O/cli_g_bf16.log 2>&1 || { tail -30 $O/cli_g_bf16.log; exit 1; }
python scripts/cli_vs_bench.py --cli $O/res/experiment_single_1_r50 --bench $O/bench.log > $O/cli_vs_bench.json
python scripts/cli_vs_bench.py --cli $O/res_fp32/experiment_single_1_gfp32 --cli $O/res_bf16/experiment_single_1_gbf16 > $O/googlenet_cli.json
grep -h img_s $O/cli_vs_bench.json $O/googlenet_cli.json | head -20
