#!/bin/bash
# Round 3, call 15: same-box interleaved A/B of the tr_frag concatenation (default _C.so vs _C_trold.so built
# with -D DLA_TR_CONCAT=0) and of the halo weight gradient (DLA_HALO_WGRAD=0), 3 rounds.
set -o pipefail
O=gpurun_out/g15; mkdir -p $O
R=$(pwd)
for i in 1 2 3; do
  for v in new trold nohalo; do
    unset DLA_EXT_SO DLA_HALO_WGRAD
    if [ $v = trold ]; then export DLA_EXT_SO=$R/distributed_learning_amd/_C_trold.so; fi
    if [ $v = nohalo ]; then export DLA_HALO_WGRAD=0; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
