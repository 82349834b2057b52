#!/bin/bash
# Round 6, call g28: counter tables of the final-tree bs1280 step (deferred block-final apply) (MFMA busy per kernel: one SQ pass; HBM-side
# bytes per kernel: FETCH_SIZE and WRITE_SIZE passes), each pass its own run
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r6/g28
mkdir -p $O
bash scripts/gpu_pmc_mfma.sh || { tail -20 gpurun_out/pmc_mfma.log; exit 1; }
mv gpurun_out/mfma_util* $O/ && mv gpurun_out/pmc_mfma.log $O/
echo "mfma pass done"
bash scripts/gpu_pmc_bench.sh || { tail -20 gpurun_out/pmcb_*.log; exit 1; }
echo "bytes passes done"
python3 scripts/pmc_bytes.py gpurun_out --steps 2 --fetch-scale 2 > $O/bytes_per_kernel_x2.md || exit 1
python3 scripts/pmc_bytes.py gpurun_out --steps 2 --by-grid > $O/bytes_per_kernel_by_grid.md || exit 1
rm -rf gpurun_out/pmcb_*
head -8 $O/mfma_util.md; head -6 $O/bytes_per_kernel_x2.md
