#!/bin/bash
# Per-kernel HBM-side traffic of the bench step: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE
# cannot share one pass), kernel-trace CSVs copied to gpurun_out/pmcb_<pass>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=$R/miopen_db
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d /tmp/pmcb_$c -o p -- python3 $R/bench.py --steps 3 --warmup 2 "$@" > $R/gpurun_out/pmcb_$c.log 2>&1 || exit $?
  mkdir -p $R/gpurun_out/pmcb_$c; find /tmp/pmcb_$c -name '*counter_collection.csv' -exec cp {} $R/gpurun_out/pmcb_$c/ \;
done
