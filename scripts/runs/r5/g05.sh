#!/bin/bash
# Round 5, call g05: BASELINE config #5 at the batch it names (ResNet-152 at per-GPU batch 1280: bucket sweep
# incl. the reference's 256 KiB point, forced multi-rank data path, reference-schema phases CSV, peak memory),
# its teacher-forced stem + stage-1 parity at that batch, and a fresh kernel trace of the ResNet-50 step
set -o pipefail
O=gpurun_out/r5/g05
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 900 python -u bench.py --model resnet152 --batch 1280 --force_comm 1 --bucket_mb_sweep 0,0.25,1,4,8,16,25,64 \
  --steps 5 --warmup 2 --phases 3 --phases_csv $O/r152_bs1280_times.csv > $O/r152_bs1280_sweep.jsonl 2> $O/r152_sweep.err \
  || { tail -20 $O/r152_sweep.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r5/g05/r152_bs1280_sweep.jsonl") if l.startswith("{")][-1])
print("r152", d["config"]["per_gpu_batch"], d["value"], d["ms_per_step"], "peak", d["peak_mem_gb"], d.get("latency_breakdown_ms"))
for r in d["bucket_sweep"]:
    print(r)
PY
export TMPDIR=/tmp
run 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 bench.py --steps 8 --warmup 3 \
  > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 7 --out $O/ksum > /dev/null || exit 1
python scripts/stream_timeline.py $O/prof/trace_results.db --steps 7 --out $O/timeline.md > /dev/null || exit 1
rm -f $O/prof/trace_results.db
head -20 $O/ksum.md
run 600 python -u scripts/parity_at_batch.py --model resnet152 --batch 1280 > $O/r152_parity.jsonl 2> $O/r152_parity.err \
  || { tail -20 $O/r152_parity.err; cat $O/r152_parity.jsonl; exit 1; }
cut -c1-600 $O/r152_parity.jsonl
