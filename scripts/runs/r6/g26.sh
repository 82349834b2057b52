#!/bin/bash
# Round 6, call g26: BASELINE config #5 (ResNet-152 at per-GPU batch 1280, bucket sweep incl. the reference's
# 256 KiB point, forced multi-rank data path, reference-schema phases CSV) and config #4 (ResNet-50 fusion off,
# strict and grouped) on the final kernels
set -o pipefail
O=gpurun_out/r6/g26
mkdir -p $O
timeout -k 10 900 python -u bench.py --model resnet152 --batch 1280 --force_comm 1 --bucket_mb_sweep 0,0.25,1,4,8,16,25,64 \
  --steps 5 --warmup 2 --phases 3 --phases_csv $O/r152_bs1280_times.csv > $O/r152_bs1280_sweep.jsonl 2> $O/r152_sweep.err \
  || { tail -20 $O/r152_sweep.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r6/g26/r152_bs1280_sweep.jsonl") if l.startswith("{")][-1])
print("r152", d["config"].get("per_gpu_batch"), d["value"], d["ms_per_step"], "peak", d.get("peak_mem_gb"), d.get("latency_breakdown_ms"))
for r in d.get("bucket_sweep", []):
    print(r)
PY
for lg in 0 1; do
  DLA_LAUNCH_GROUPS=$lg timeout -k 10 400 python bench.py --batch 1280 --force_comm 1 --bucket_mb 0 --steps 10 --warmup 3 \
    --phases 3 --phases_csv $O/r50_fusion_off_lg$lg.csv > $O/r50_fusion_off_lg$lg.jsonl 2> $O/r50_lg$lg.err || { tail $O/r50_lg$lg.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/r50_fusion_off_lg$lg.jsonl').read().strip().splitlines()[-1]); print('r50 fusion off lg$lg', d['value'], d['ms_per_step'], d.get('fusion_off'), d.get('collectives_per_step'), d.get('launch_units_per_step'))"
done
