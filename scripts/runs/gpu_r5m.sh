#!/bin/bash
# final-state check: full GPU suite + smoke + default bench, then the step's kernel-trace summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash scripts/gpu_full.sh || exit 1
bash scripts/gpu_bench_prof.sh r5m || { tail -20 gpurun_out/prof_r5m.log; exit 1; }
head -22 gpurun_out/ksum_r5m.md
