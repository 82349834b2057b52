#!/bin/bash
# Round 3, call 10: per-kernel HBM bytes at ResNet-50 bs1024: two rocprofv3 --pmc
# passes (FETCH_SIZE, WRITE_SIZE; they cannot share a pass) joined into an achieved-TB/s table, by
# kernel and by (kernel, grid) to separate the layers of one template.
set -o pipefail
O=gpurun_out/g10; mkdir -p $O
timeout -k 10 700 bash scripts/gpu_pmc_bench.sh > $O/pmc.log 2>&1 || { tail -30 $O/pmc.log; tail -20 gpurun_out/pmcb_*.log; exit 1; }
python3 scripts/pmc_bytes.py gpurun_out --steps 2 > $O/bytes_table.md
python3 scripts/pmc_bytes.py gpurun_out --steps 2 --by-grid --top 120 > $O/bytes_by_grid.md
head -40 $O/bytes_table.md
