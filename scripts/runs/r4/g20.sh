#!/bin/bash
# Round 4, call g20: the g03 gradient-path records again on the final kernels (one-pass 1x1 gradients + fused
# block-final BN apply): forced-comm A/B, final-step kernel summary, fusion off / on with the reference's
# latency-breakdown columns, ResNet-152 bucket sweep
set -o pipefail
O=gpurun_out/g20
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_default.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u bench.py --steps 15 --warmup 5 --force_comm 1 >> $O/ab_force.jsonl 2>> $O/ab.err || exit 1
done
export TMPDIR=/tmp
run 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 bench.py --steps 8 --warmup 3 \
  > $O/prof.log 2>&1 || exit 1
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 7 --out $O/ksum_final > /dev/null || exit 1
python scripts/stream_timeline.py $O/prof/trace_results.db --steps 7 --out $O/timeline_final.md > /dev/null || exit 1
rm -f $O/prof/trace_results.db
run 300 python -u bench.py --force_comm 1 --bucket_mb 0 --steps 10 --warmup 3 --phases 5 \
  --phases_csv $O/fusion_off_times.csv > $O/fusion_off.jsonl 2> $O/fusion_off.err || exit 1
run 300 python -u bench.py --force_comm 1 --steps 10 --warmup 3 --phases 5 \
  --phases_csv $O/fusion_on_times.csv > $O/fusion_on.jsonl 2> $O/fusion_on.err || exit 1
run 600 python -u bench.py --model resnet152 --batch 256 --force_comm 1 --bucket_mb_sweep 0,1,4,8,16,25,64 \
  --steps 10 --warmup 3 > $O/r152_sweep.jsonl 2> $O/r152_sweep.err || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/g20/*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], d.get("value"), d.get("ms_per_step"), d.get("config", {}).get("bucket_mb"))
PY
