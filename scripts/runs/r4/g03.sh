#!/bin/bash
# Round 4, call g03: the gradient path at the shipped configuration.
#  1. --force_comm 1 vs 0 at the default batch (1280), interleaved: the per-GPU cost of the N > 1 data path
#     (gather -> fp32 staging -> collective -> cast) with the autotuner's table at world 1
#  2. a rocprofv3 kernel trace of the forced run -> per-stream timeline (scripts/stream_timeline.py)
#  3. fusion off (--bucket_mb 0, one collective per tensor) with the reference's latency-breakdown columns
#  4. ResNet-152 bucket sweep 1..64 MiB (the reference's fusion_experiment), forced 1-rank collectives
set -o pipefail
O=gpurun_out/g03
mkdir -p $O
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
run() { timeout -k 10 "$1" "${@:2}"; }
for i in 1 2; do
  run 200 python -u bench.py --steps 15 --warmup 5 >> $O/ab_default.jsonl 2>> $O/ab.err || exit 1
  run 200 python -u bench.py --steps 15 --warmup 5 --force_comm 1 >> $O/ab_force.jsonl 2>> $O/ab.err || exit 1
done
export TMPDIR=/tmp
run 400 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 bench.py --steps 8 --warmup 3 --force_comm 1 \
  > $O/prof.log 2>&1 || exit 1
run 300 python -u bench.py --force_comm 1 --bucket_mb 0 --steps 10 --warmup 3 --phases 5 \
  --phases_csv $O/fusion_off_times.csv > $O/fusion_off.jsonl 2> $O/fusion_off.err || exit 1
run 300 python -u bench.py --force_comm 1 --steps 10 --warmup 3 --phases 5 \
  --phases_csv $O/fusion_on_times.csv > $O/fusion_on.jsonl 2> $O/fusion_on.err || exit 1
run 400 python -u bench.py --gpus 2 --same_device 1 --batch 256 --steps 10 --warmup 3 \
  > $O/two_ranks_one_gpu.jsonl 2> $O/two_ranks_one_gpu.err || exit 1
run 600 python -u bench.py --model resnet152 --batch 256 --force_comm 1 --bucket_mb_sweep 0,1,4,8,16,25,64 \
  --steps 10 --warmup 3 > $O/r152_sweep.jsonl 2> $O/r152_sweep.err || exit 1
