#!/bin/bash
# Round 3, call 24: replay difference with the late 3x3 weight gradients (no DP wrapper): explicit join after
# backward, device drain after backward, caching allocator off.
set -o pipefail
O=gpurun_out/g24; mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 90 python3 scripts/race_replay.py /tmp/$tag.conc.pt > $O/$tag.conc.log 2>&1 || { tail -20 $O/$tag.conc.log; return 1; }
  env "$@" AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 90 python3 scripts/race_replay.py /tmp/$tag.ser.pt > $O/$tag.ser.log 2>&1 || { tail -20 $O/$tag.ser.log; return 1; }
  echo "$tag: $(python3 scripts/race_compare.py /tmp/$tag.conc.pt /tmp/$tag.ser.pt)" | tee -a $O/summary.txt
  python3 scripts/race_compare.py /tmp/$tag.conc.pt /tmp/defer0.ser.pt | sed "s/^/  conc vs defer0.ser: /" | tee -a $O/summary.txt
}
run defer0 DLA_WGRAD_DEFER=0 RACE_NODP=1 || exit 1
run plain DLA_WGRAD_DEFER=3x3 RACE_NODP=1 || exit 1
run join DLA_WGRAD_DEFER=3x3 RACE_NODP=1 RACE_JOIN=1 || exit 1
run sync DLA_WGRAD_DEFER=3x3 RACE_NODP=1 RACE_SYNC=1 || exit 1
run nocache DLA_WGRAD_DEFER=3x3 RACE_NODP=1 PYTORCH_NO_CUDA_MEMORY_CACHING=1 || exit 1
