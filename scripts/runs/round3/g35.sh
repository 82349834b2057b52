#!/bin/bash
# Round 3, call 35: BN-backward finalize capped at 32 VGPRs (fits beside a 256x256 weight-gradient block,
# so the late weight gradients do not hold it back) vs the 8-in-flight uncapped finalize (_C_fin8.so);
# BN numerics tests, then 3 interleaved rounds and a kernel profile of the new default.
set -o pipefail
O=gpurun_out/g35; mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn_act.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2 3; do
  for v in lean fin8; do
    unset DLA_EXT_SO
    if [ $v = fin8 ]; then export DLA_EXT_SO=$R/distributed_learning_amd/_C_fin8.so; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
unset DLA_EXT_SO
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g35prof -o prof -- python3 $R/bench.py --steps 20 --warmup 5 > $R/$O/prof.log 2>&1 || { tail -30 $R/$O/prof.log; exit 1; }
cd $R
T=$(find /tmp/g35prof -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 20 --out $O/ksum > /dev/null
sed -n 3,6p $O/ksum.md; grep "bn_bwd_finalize\|bn_bwd_apply_kernel<unsigned short, 1" $O/ksum.md
