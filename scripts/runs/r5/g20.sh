#!/bin/bash
# Round 5, call g20: counter tables of the shipped bs1280 step (verdict r4 item 2): MFMA busy per kernel (one
# SQ pass), HBM-side bytes per kernel (FETCH_SIZE and WRITE_SIZE passes), and a --stats run for durations
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r5/g20
mkdir -p $O
bash scripts/gpu_pmc_mfma.sh || { tail -20 gpurun_out/pmc_mfma.log; exit 1; }
mv gpurun_out/mfma_util* $O/ && mv gpurun_out/pmc_mfma.log $O/
bash scripts/gpu_pmc_bench.sh || { tail -20 gpurun_out/pmcb_*.log; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/st -o s -- python3 $R/bench.py --steps 3 --warmup 2 \
  > $O/stats.log 2>&1 || { tail $O/stats.log; exit 1; }
find /tmp/st -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
python3 scripts/pmc_bytes.py gpurun_out --steps 2 > $O/bytes_per_kernel.md || exit 1
python3 scripts/pmc_bytes.py gpurun_out --steps 2 --by-grid > $O/bytes_per_kernel_by_grid.md || exit 1
rm -rf gpurun_out/pmcb_*
head -8 $O/mfma_util.md; head -12 $O/bytes_per_kernel.md
