#!/bin/bash
# Round 3, call 42: final-state counters: MFMA utilisation per kernel (one pass) and per-kernel HBM bytes
# (FETCH_SIZE / WRITE_SIZE passes), each its own rocprofv3 run; tables under gpurun_out/.
set -o pipefail
R=$(pwd)
timeout -k 10 360 bash scripts/gpu_pmc_mfma.sh || exit 1
head -12 gpurun_out/mfma_util.md
timeout -k 10 700 bash scripts/gpu_pmc_bench.sh || exit 1
python3 scripts/pmc_bytes.py gpurun_out --fetch-scale 2 > gpurun_out/bytes_table.md 2>&1 || { tail -5 gpurun_out/bytes_table.md; exit 1; }
head -14 gpurun_out/bytes_table.md
