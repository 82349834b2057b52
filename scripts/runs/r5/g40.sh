#!/bin/bash
# Round 5, call g40: where the step's ~200 memsets and ~165 device copies per step come from (torch profiler,
# tables by CUDA time and by call count with Python stacks)
set -o pipefail
O=gpurun_out/r5/g40
mkdir -p $O
DLA_TORCH_PROF=$O/torch_prof.txt timeout -k 10 400 python bench.py --steps 5 --warmup 3 > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep -n -i -E "memset|memcpy|aten::copy_|aten::zero_|aten::fill_|aten::zeros" $O/torch_prof.txt | head -40
