#!/bin/bash
# Round 6, call g27: side-stream scheduling re-checked on the final step -- driver bench per setting, interleaved x2
set -o pipefail
O=gpurun_out/r6/g27
mkdir -p $O
run() {  # tag, env assignments...
  local t=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/$t.jsonl 2>> $O/err.log || { echo "$t failed"; tail $O/err.log; exit 1; }
}
for i in 1 2; do
  run base DLA_NOOP=1
  run defer_all DLA_WGRAD_DEFER=all
  run join_conv DLA_WGRAD_JOIN=conv
  run defer_off DLA_WGRAD_DEFER=0
  echo "round $i done"
done
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r6/g27/*.jsonl")):
    v = [json.loads(l) for l in open(f) if l.startswith("{")]
    print(os.path.basename(f)[:-6], [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
