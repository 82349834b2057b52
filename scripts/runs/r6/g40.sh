#!/bin/bash
# Round 6, call g40: the register-direct epilogue shared (dla_mfma.h epilogue_direct with an optional addend now also
# serves the halo data gradient; gemm_direct uses the shared DPP row sum) -- tests, driver bench x2
set -o pipefail
O=gpurun_out/r6/g40
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_gemm_direct.py tests/test_gpu_gemm256_direct.py -x -q --timeout 200 --timeout-method thread > $O/test.txt 2>&1 || { grep -E "Error|assert|FAIL" $O/test.txt | head; tail -30 $O/test.txt; exit 1; }
tail -1 $O/test.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O/bench.jsonl 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
python3 -c "
import json
for l in open('$O/bench.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'], d['telemetry']['before_timed']['gfxclk_mhz'])"
