#!/bin/bash
# Round 3, call 44: main loop of the 128-row-tile 1x1 GEMMs with K <= 512 at bs1024 (the r2t A/B chose
# register staging at bs512, before the buffer-DMA loop): DLA_NT_PIPE unset (0) vs 6 / 2 / 4; 2 rounds.
set -o pipefail
O=gpurun_out/g44; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for v in def 6 2 4; do
    unset DLA_NT_PIPE
    if [ $v != def ]; then export DLA_NT_PIPE=$v; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${v}_$i.log 2>&1 || { tail -30 $O/bench_${v}_$i.log; exit 1; }
    echo "nt_pipe=$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)" | tee -a $O/ab.txt
  done
done
