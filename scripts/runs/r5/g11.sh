#!/bin/bash
# Round 5, call g11: the stem BN+ReLU+max-pool backward apply fused into the stem weight gradient -- numerics
# (vs the unfused pair and fp32 PyTorch), the stem op alone fused vs unfused, the bs256 step A/B interleaved x3,
# and a kernel trace of the fused step
set -o pipefail
O=gpurun_out/r5/g11
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u -m pytest tests/test_gpu_stem_bn_fused.py tests/test_gpu_stem.py -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/test.log | tail -15
run 200 python -u scripts/bench_stem.py > $O/stem_fused.jsonl 2> $O/stem.err || { tail $O/stem.err; exit 1; }
DLA_STEM_BN=0 run 200 python -u scripts/bench_stem.py > $O/stem_unfused.jsonl 2>> $O/stem.err || { tail $O/stem.err; exit 1; }
cat $O/stem_fused.jsonl $O/stem_unfused.jsonl | cut -c1-400
for i in 1 2 3; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_fused.jsonl 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
  DLA_STEM_BN=0 run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_unfused.jsonl 2>> $O/ab.err \
    || { tail $O/ab.err; exit 1; }
done
python - <<'PY'
import json
for k in ("fused", "unfused"):
    v = [json.loads(l) for l in open(f"gpurun_out/r5/g11/ab_{k}.jsonl") if l.startswith("{")]
    print(k, [round(d["value"]) for d in v], [round(d["ms_per_step"], 2) for d in v], v[-1].get("knobs"))
PY
export TMPDIR=/tmp
run 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 bench.py --steps 8 --warmup 3 \
  > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 7 --out $O/ksum > /dev/null || exit 1
rm -f $O/prof/trace_results.db
head -24 $O/ksum.md
