#!/bin/bash
# PMC pass over the max-pool microbenchmark (is the 3x3/s1 pool VALU- or memory-bound?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out/r3t; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d /tmp/pm_pool -o p -- python3 $R/scripts/pool_probe.py --iters 5 > $R/gpurun_out/r3t/pmc.log 2>&1 || { tail -5 $R/gpurun_out/r3t/pmc.log; exit 1; }
find /tmp/pm_pool -name '*counter_collection.csv' -exec cp {} $R/gpurun_out/r3t/ \;
python3 $R/scripts/pmc_table.py $R/gpurun_out/r3t/*counter_collection.csv --match maxpool > $R/gpurun_out/r3t/table.txt 2>&1
cat $R/gpurun_out/r3t/table.txt | head -20
