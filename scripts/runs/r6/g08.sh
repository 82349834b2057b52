#!/bin/bash
# Round 6, call g08: fp32 Inception fan-in (three 1x1 convs on x as one GEMM, one BN pass) -- tests, fp32 GoogLeNet
# line, fp32 path accuracy test, kernel trace of the fp32 step
set -o pipefail
O=gpurun_out/r6/g08
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_f32.py tests/test_gpu_inception_f32.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp32_path.py -x -v -s --timeout 300 --timeout-method thread > $O/fp32_path.txt 2>&1 || { tail -30 $O/fp32_path.txt; exit 1; }
grep -E "vs fp64|PASSED|FAILED" $O/fp32_path.txt | cut -c1-300
export MIOPEN_USER_DB_PATH=$(pwd)/miopen_db
timeout -k 10 300 python bench.py --model googlenet --precision fp32 --batch 128 --steps 20 --warmup 5 > $O/gnet_fp32.jsonl 2> $O/gnet.err || { tail $O/gnet.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/gnet_fp32.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['conv1x1'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 bench.py --model googlenet --precision fp32 --batch 128 \
  --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python scripts/kernel_summary.py $O/prof/trace_results.db --steps 7 --out $O/ksum_gnet_fp32 > /dev/null || exit 1
rm -f $O/prof/trace_results.db
head -50 $O/ksum_gnet_fp32.md
