#!/bin/bash
# Round 3, call 22: race-replay diagnosis of the g20 failure (concurrent vs serialised run differ with the
# late-joined 3x3 weight gradients on): defer off / on, halo weight gradient off, no DP wrapper.
set -o pipefail
O=gpurun_out/g22; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 60 python3 scripts/race_replay.py $O/$tag.conc.pt > $O/$tag.conc.log 2>&1 || { tail -20 $O/$tag.conc.log; return 1; }
  env "$@" AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 60 python3 scripts/race_replay.py $O/$tag.ser.pt > $O/$tag.ser.log 2>&1 || { tail -20 $O/$tag.ser.log; return 1; }
  echo "$tag: $(python3 scripts/race_compare.py $O/$tag.conc.pt $O/$tag.ser.pt)" | tee -a $O/summary.txt
}
run defer0 DLA_WGRAD_DEFER=0 || exit 1
run defer3x3 DLA_WGRAD_DEFER=3x3 || exit 1
run defer3x3_b DLA_WGRAD_DEFER=3x3 || exit 1
run defer3x3_nohalo DLA_WGRAD_DEFER=3x3 DLA_HALO_WGRAD=0 || exit 1
run defer3x3_joinconv DLA_WGRAD_DEFER=3x3 DLA_WGRAD_JOIN=conv || exit 1
run defer3x3_nodp DLA_WGRAD_DEFER=3x3 RACE_NODP=1 || exit 1
