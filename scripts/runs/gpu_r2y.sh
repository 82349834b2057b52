#!/bin/bash
# refreshed ResNet-50 bs512 step profile (kernel trace) + per-kernel HBM bytes (FETCH/WRITE_SIZE)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_bench_prof.sh r2y || exit 1
head -70 $R/gpurun_out/ksum_r2y.md
bash $R/scripts/gpu_pmc_bench.sh || exit 1
cd $R && python3 scripts/pmc_bytes.py gpurun_out 3 > gpurun_out/r2y_bytes.md 2>&1; head -45 gpurun_out/r2y_bytes.md
