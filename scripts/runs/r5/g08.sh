#!/bin/bash
# Round 5, call g08: the reference-precision path (fp32 GoogLeNet) on the native BN/pool/loss/SGD kernels:
# parity test against stock fp32 PyTorch, the bench at batch 128 (stock NCHW vs native, eager and HIP graph), and
# its kernel summary
set -o pipefail
O=gpurun_out/r5/g08
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u -m pytest tests/test_gpu_fp32_path.py -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider \
  > $O/test.log 2>&1; grep -E "worst gradients|median gradient" $O/test.log | cut -c1-1500
grep -E "PASSED|FAILED" $O/test.log
export MIOPEN_USER_DB_PATH=$(pwd)/miopen_db
for k in torch native; do
  run 300 python -u bench.py --model googlenet --precision fp32 --batch 128 --kernels $k --steps 20 --warmup 5 \
    > $O/gnet_fp32_$k.jsonl 2> $O/gnet_fp32_$k.err || { tail $O/gnet_fp32_$k.err; exit 1; }
done
run 400 python -u bench.py --model googlenet --precision fp32 --batch 128 --kernels native --graph on --steps 20 --warmup 5 \
  > $O/gnet_fp32_native_graph.jsonl 2> $O/gnet_fp32_native_graph.err || { tail $O/gnet_fp32_native_graph.err; exit 1; }
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5/g08/gnet*.jsonl")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["vs_baseline"], d["config"]["kernels"], d["config"].get("layout"), d["config"]["hip_graph"])
PY
export TMPDIR=/tmp
run 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 bench.py --model googlenet --precision fp32 --batch 128 \
  --kernels native --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 7 --out $O/ksum_gnet_fp32 > /dev/null || exit 1
rm -f $O/prof/trace_results.db
head -24 $O/ksum_gnet_fp32.md
