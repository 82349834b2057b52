#!/bin/bash
# Round 5, call g06: where the 3x3 convs and the stem lose time at bs1280 -- per-tile timing of every 3x3 shape,
# the stem op alone (+ its kernel trace), and one PMC pass over the 3x3 micro-benchmark (MFMA busy, LDS
# bank conflicts / unaligned stalls, VALU and LDS instruction counts)
set -o pipefail
O=gpurun_out/r5/g06
mkdir -p $O
run() { timeout -k 10 "$1" "${@:2}"; }
run 300 python -u scripts/bench_conv_tiles.py > $O/conv_tiles.jsonl 2> $O/conv_tiles.err || { tail $O/conv_tiles.err; exit 1; }
cat $O/conv_tiles.jsonl
run 200 python -u scripts/bench_stem.py > $O/stem.jsonl 2> $O/stem.err || { tail $O/stem.err; exit 1; }
cat $O/stem.jsonl
export TMPDIR=/tmp
R=$(pwd)
run 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/stemprof -o s -- python3 $R/scripts/bench_stem.py --iters 10 \
  > $O/stem_prof.log 2>&1 || { tail $O/stem_prof.log; exit 1; }
find /tmp/stemprof -name '*kernel_stats.csv' -exec cp {} $O/stem_kernel_stats.csv \;
head -20 $O/stem_kernel_stats.csv | cut -c1-200
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL \
  SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d /tmp/convpmc -o c -- \
  python3 $R/scripts/bench_conv_tiles.py > $O/conv_pmc.log 2>&1 || { tail $O/conv_pmc.log; exit 1; }
find /tmp/convpmc -name '*counter_collection.csv' -exec cp {} $O/conv_pmc.csv \;
ls -la $O
