#!/bin/bash
# Round 6, call g41: round-end sequence on the final tree (after the g40 epilogue refactor) (full GPU suite, smoke,
# driver bench x2) and a kernel trace of the bf16 ResNet-50 bs1280 step
set -o pipefail
O=gpurun_out/r6/g41
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread > $O/full_gpu.log 2>&1 || { echo "GPU suite failed"; grep -E "Error|assert|FAIL|failed" $O/full_gpu.log | head -20; tail -30 $O/full_gpu.log; exit 1; }
tail -2 $O/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-300
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/bench.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'], d['telemetry']['before_timed'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 bench.py --steps 4 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 3 --out $O/ksum > /dev/null || exit 1
rm -f $O/prof/trace_results.db
head -45 $O/ksum.md
