#!/bin/bash
# Round 3, call 18: late-joined weight gradients (ops/conv.py WGRAD_DEFER): bitwise tests, then an
# interleaved end-to-end A/B of the defer / join modes, 2 rounds.
set -o pipefail
O=gpurun_out/g18; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wgrad_defer.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  for v in 0:end 3x3:end all:end 3x3:conv all:conv; do
    d=${v%%:*}; j=${v##*:}
    DLA_WGRAD_DEFER=$d DLA_WGRAD_JOIN=$j timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_${d}_${j}_$i.log 2>&1 || { tail -30 $O/bench_${d}_${j}_$i.log; exit 1; }
    echo "defer=$d join=$j $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${d}_${j}_$i.log) peak $(grep -o '"peak_mem_gb": [0-9.]*' $O/bench_${d}_${j}_$i.log)" | tee -a $O/ab.txt
  done
done
