#!/bin/bash
# Round 6, call g04: strict fusion-off (DLA_LAUNCH_GROUPS=0, one collective launch per gradient tensor; verdict r5
# item 3) vs the grouped form -- GPU test, then ResNet-50 / ResNet-152 at bs256 and bs1280, forced world-1 data path,
# --bucket_mb 0 with reference-schema phase CSVs; then the 2-rank same-device N>1 line with autotune_s (items 4, 6)
set -o pipefail
O=gpurun_out/r6/g04
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 600 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fusion_off" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED" $O/tests.log
for cfg in "resnet50 256" "resnet50 1280" "resnet152 256" "resnet152 1280"; do
  set -- $cfg
  for lg in 0 1; do
    tag=${1}_bs${2}_lg${lg}
    DLA_LAUNCH_GROUPS=$lg run 400 python -u bench.py --model $1 --batch $2 --force_comm 1 --bucket_mb 0 --steps 10 --warmup 3 \
      --phases 5 --phases_csv $O/${tag}_times.csv > $O/${tag}.jsonl 2> $O/${tag}.err || { tail $O/${tag}.err; exit 1; }
    echo "$tag done"
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6/g04/*.jsonl")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], d["value"], d["ms_per_step"], "comm", d.get("allreduce_ms_per_step"), d.get("fusion_off"),
                  "coll/step", d.get("collectives_per_step"), "launch/step", d.get("launch_units_per_step"))
PY
export DLA_COMM_TIMEOUT_S=60
run 400 python bench.py --gpus 2 --same_device 1 --batch 64 --steps 4 --warmup 2 > $O/bench2.log 2>&1 || { tail -30 $O/bench2.log; exit 1; }
grep metric $O/bench2.log > $O/bench2.jsonl
python -c "import json; d=json.loads(open('$O/bench2.jsonl').read()); print(d['value'], d['n_gpus'], d['comm_world'], d['comm_world_src'], 'autotune_s', d.get('autotune_s'), d['allreduce_per_bucket'][:8], d['allreduce_table'].get('excluded'))"
