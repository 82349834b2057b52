#!/bin/bash
# per-layer sweeps: tile config (fwd/dgrad), main loop 2/4/6, split-K block target (wgrad)
set -o pipefail
mkdir -p gpurun_out/r2v
for t in 0 1 2 3; do
  timeout -k 10 300 python scripts/bench_layers.py --only fwd,dgrad --tile $t --out gpurun_out/r2v/tile$t.jsonl > gpurun_out/r2v/tile$t.log 2>&1 || { tail -5 gpurun_out/r2v/tile$t.log; exit 1; }
  echo "tile=$t"; grep -A6 "conv time" gpurun_out/r2v/tile$t.log
done
for p in 2 4 6; do
  timeout -k 10 300 python scripts/bench_layers.py --pipe $p --out gpurun_out/r2v/pipe$p.jsonl > gpurun_out/r2v/pipe$p.log 2>&1 || { tail -5 gpurun_out/r2v/pipe$p.log; exit 1; }
  echo "pipe=$p"; grep -A8 "conv time" gpurun_out/r2v/pipe$p.log | grep 3x3
done
for b in 256 512 1024 2048; do
  DLA_SPLITK_BLOCKS=$b timeout -k 10 300 python scripts/bench_layers.py --only wgrad --out gpurun_out/r2v/wg$b.jsonl > gpurun_out/r2v/wg$b.log 2>&1 || { tail -5 gpurun_out/r2v/wg$b.log; exit 1; }
  echo "splitk_blocks=$b"; grep -A4 "conv time" gpurun_out/r2v/wg$b.log
done
