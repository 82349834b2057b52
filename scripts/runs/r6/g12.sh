#!/bin/bash
# Round 6, call g12: the round-end sequence on the current tree (full GPU suite, smoke, driver bench) plus the fp32
# GoogLeNet line eager and under HIP-graph replay
set -o pipefail
O=gpurun_out/r6/g12
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread > $O/full_gpu.log 2>&1 || { echo "GPU suite failed"; grep -E "Error|assert|FAIL|failed" $O/full_gpu.log | head -20; tail -30 $O/full_gpu.log; exit 1; }
tail -2 $O/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-300
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['telemetry']['before_timed'])"
export MIOPEN_USER_DB_PATH=$(pwd)/miopen_db
for gm in off on; do
  timeout -k 10 400 python bench.py --model googlenet --precision fp32 --batch 128 --graph $gm --steps 20 --warmup 5 > $O/gnet_fp32_graph_$gm.jsonl 2> $O/gnet_$gm.err || { tail $O/gnet_$gm.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/gnet_fp32_graph_$gm.jsonl').read().strip().splitlines()[-1]); print('graph $gm', d['value'], d['ms_per_step'], d['config']['conv1x1'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 bench.py --model googlenet --precision fp32 --batch 128 \
  --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 7 --out $O/ksum_gnet_fp32 > /dev/null || exit 1
rm -f $O/prof/trace_results.db
head -24 $O/ksum_gnet_fp32.md
grep -E "igemm|SubTensor|stem|Cijk" $O/ksum_gnet_fp32.md | cut -c1-160
