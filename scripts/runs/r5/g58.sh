#!/bin/bash
# Round 5, call g58: round-end sequence on the final tree (after the stride-2 512x128 data gradient) -- full GPU suite, smoke,
# driver bench command x2, then a kernel-trace of 3 steady-state steps summarised per kernel
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r5/g58
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/full_gpu.log 2>&1 || { echo "GPU suite failed"; grep -E "Error|assert|FAIL|failed" $O/full_gpu.log | head -20; tail -30 $O/full_gpu.log; exit 1; }
tail -2 $O/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
done
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench.jsonl
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt -o s -- python3 $R/bench.py --steps 4 --warmup 2 \
  > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
T=$(find /tmp/kt -name '*kernel_trace.csv' | head -1)
python3 scripts/kernel_summary.py "$T" --steps 3 --out $O/ksum > $O/ksum.txt 2>&1 || { tail $O/ksum.txt; exit 1; }
head -30 $O/ksum.txt
