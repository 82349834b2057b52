#!/bin/bash
# halo conv variant 2 (VGPR weights, two blocks per CU): tests, per-layer A/B of v1 / v2 / off
# (forward + dgrad routed, DLA_HALO=2), whole-step A/B
set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j/conv_tests.log 2>&1 || { tail -40 gpurun_out/r5j/conv_tests.log; exit 1; }
tail -1 gpurun_out/r5j/conv_tests.log
sed 's/\["1"\])  # variant 2/["1", "2"])  # variant 2/' tests/test_gpu_conv3x3.py > tests/_halo_v2_check.py && timeout -k 10 300 python -u -m pytest tests/_halo_v2_check.py -x -q -k halo --timeout 240 --timeout-method thread > gpurun_out/r5j/halo_v2_test.log 2>&1 || { tail -40 gpurun_out/r5j/halo_v2_test.log; exit 1; }
tail -1 gpurun_out/r5j/halo_v2_test.log
for r in 1 2; do
  for v in 0 1 2; do
    if [ $v = 0 ]; then H=0; V=2; else H=2; V=$v; fi
    DLA_HALO=$H DLA_HALO_V=$V timeout -k 10 240 python -u scripts/bench_layers.py --only fwd,dgrad --out gpurun_out/r5j/layers_v${v}_r$r.jsonl > gpurun_out/r5j/layers.log 2>&1 || { tail -20 gpurun_out/r5j/layers.log; exit 1; }
  done
done
grep s56_c2 gpurun_out/r5j/layers_v*_r*.jsonl | cut -c1-200
for i in 1 2; do
  for cfg in "2 2" "2 1" "1 1" "0 1"; do
    set -- $cfg
    DLA_HALO=$1 DLA_HALO_V=$2 timeout -k 10 300 python bench.py > gpurun_out/r5j/bench_h$1v$2_${i}.log 2>&1 || { tail -20 gpurun_out/r5j/bench_h$1v$2_${i}.log; exit 1; }
    echo "halo=$1 v=$2 $(grep -o '"value": [0-9.]*' gpurun_out/r5j/bench_h$1v$2_${i}.log | head -1)" | tee -a gpurun_out/r5j/ab.txt
  done
done
bash scripts/gpu_full.sh
