#!/bin/bash
# Round 3, call 7: streaming virtual-y kernels with buffer-op loads/stores and ping-pong registers:
# unit tests, A/B bench (DLA_VIRTUAL_Y 1 vs 0), kernel profile.
set -o pipefail
O=gpurun_out/g07; mkdir -p $O
R=$(pwd)
PT="python -u -m pytest -x -v -s --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_virtual_y.py > $O/pytest_vy.log 2>&1 || { tail -60 $O/pytest_vy.log; exit 1; }
tail -2 $O/pytest_vy.log
for i in 1 2; do
  for v in 1 0; do
    DLA_VIRTUAL_Y=$v timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_vy${v}_$i.log 2>&1 || { tail -30 $O/bench_vy${v}_$i.log; exit 1; }
    echo "vy=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_vy${v}_$i.log)" | tee -a $O/ab.txt
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/g07prof -o prof -- python3 $R/bench.py --gpus 1 --steps 8 --warmup 4 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
T=$(find /tmp/g07prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 8 --out $O/ksum > /dev/null
grep -E "vy_stream|batchnorm|gemm \|" $O/ksum.md | head -20
