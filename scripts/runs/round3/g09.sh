#!/bin/bash
# Round 3, call 9: GEMM-epilogue addend preload (all rows' D / mask / d2 loads issued before the store
# loop) vs the per-row loads (variant build _C_nopre.so): GEMM/conv/BN-epilogue tests, interleaved A/B,
# kernel profile of the new default; plus DLA_BN_EPILOGUE=1 (BN-backward reduce folded into the consumer
# conv dgrad epilogue, 0.3 ms slower at bs512 before the preload).
set -o pipefail
O=gpurun_out/g09; mkdir -p $O
R=$(pwd)
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_gemm.py tests/test_gpu_bn_epilogue.py tests/test_gpu_conv.py tests/test_gpu_conv3x3.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for v in pre nopre bnepi; do
    unset DLA_BN_EPILOGUE
    if [ $v = nopre ]; then export DLA_EXT_SO=$R/distributed_learning_amd/_C_nopre.so; else unset DLA_EXT_SO; fi
    if [ $v = bnepi ]; then export DLA_BN_EPILOGUE=1; fi
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
unset DLA_EXT_SO DLA_BN_EPILOGUE
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/g09prof -o prof -- python3 $R/bench.py --gpus 1 --steps 8 --warmup 4 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
T=$(find /tmp/g09prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 8 --out $O/ksum > /dev/null
sed -n 5,30p $O/ksum.md
