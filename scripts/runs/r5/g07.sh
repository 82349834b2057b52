#!/bin/bash
# Round 5, call g07: (1) A/B of the step on a high-priority compute stream (the late 3x3 weight gradients' side
# stream stays at normal priority) vs the default, interleaved x3; (2) the fused BN passes alone at the stage-1
# shapes (training apply with the 1-bit mask vs the eval apply without, backward reduce + apply)
set -o pipefail
O=gpurun_out/r5/g07
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_default.jsonl 2>> $O/ab.err || exit 1
  DLA_COMPUTE_STREAM=high timeout -k 10 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_high.jsonl 2>> $O/ab.err || exit 1
done
python - <<'PY'
import json
for f in ("ab_default", "ab_high"):
    v = [json.loads(l) for l in open(f"gpurun_out/r5/g07/{f}.jsonl") if l.startswith("{")]
    print(f, [d["value"] for d in v], [d["step_ms"]["p50"] for d in v])
PY
timeout -k 10 200 python -u scripts/bench_bn.py > $O/bn.jsonl 2> $O/bn.err || { tail $O/bn.err; exit 1; }
cat $O/bn.jsonl
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bnprof -o b -- python3 $R/scripts/bench_bn.py --iters 10 \
  > $O/bn_prof.log 2>&1 || { tail $O/bn_prof.log; exit 1; }
find /tmp/bnprof -name '*kernel_stats.csv' -exec cp {} $O/bn_kernel_stats.csv \;
cut -c1-220 $O/bn_kernel_stats.csv | head -14
