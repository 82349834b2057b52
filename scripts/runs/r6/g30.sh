#!/bin/bash
# Round 6, call g30: multiply-shift tap masks in the stage-1 halo conv (DLA_HALO_FASTDIV) -- halo tests, isolated
# kernel times (kernel trace) fwd / dgrad at bs1280, driver bench interleaved x3
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r6/g30
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv3x3.py -x -q -k "halo" --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
export CONV_ONE_N=1280
cd /tmp && export TMPDIR=/tmp
for f in 0 1; do
  for op in fwd dgrad; do
    DLA_HALO_FASTDIV=$f timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_${op}_$f -o k -- python3 $R/scripts/conv_one.py $op 64 56 64 1 20 > $O/kt_${op}_$f.log 2>&1 || { tail -5 $O/kt_${op}_$f.log; exit 1; }
    echo "fastdiv=$f $op: $(grep -h halo $(find /tmp/kt_${op}_$f -name '*kernel_stats.csv' | head -1) | cut -d, -f1-5 | cut -c1-160)"
  done
done | tee $O/isolated.txt
cd $R
for i in 1 2 3; do
  for f in 0 1; do
    DLA_HALO_FASTDIV=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/b$f.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for k in (0, 1):
    v = [json.loads(l) for l in open(f"gpurun_out/r6/g30/b{k}.jsonl") if l.startswith("{")]
    print("fastdiv", k, [round(d["value"]) for d in v], [d["ms_per_step"] for d in v],
          [d["telemetry"]["before_timed"]["gfxclk_mhz"] for d in v])
PY
