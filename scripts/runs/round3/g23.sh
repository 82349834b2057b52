#!/bin/bash
# Round 3, call 23: is the g20/g22 replay difference an intra-kernel race exposed by co-running (the late
# weight gradients overlap other kernels), or a stream-ordering bug? Co-run determinism of the 3x3 weight
# gradient kernels, then replay pairs with the halo weight gradient on / off.
set -o pipefail
O=gpurun_out/g23; mkdir -p $O
timeout -k 10 120 python3 scripts/corun_determinism.py --reps 15 > $O/corun.log 2>&1 || { tail -20 $O/corun.log; exit 1; }
cat $O/corun.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 60 python3 scripts/race_replay.py /tmp/$tag.conc.pt > $O/$tag.conc.log 2>&1 || { tail -20 $O/$tag.conc.log; return 1; }
  env "$@" AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 timeout -k 10 60 python3 scripts/race_replay.py /tmp/$tag.ser.pt > $O/$tag.ser.log 2>&1 || { tail -20 $O/$tag.ser.log; return 1; }
  echo "$tag: $(python3 scripts/race_compare.py /tmp/$tag.conc.pt /tmp/$tag.ser.pt)" | tee -a $O/summary.txt
}
for i in 1 2 3; do
  run nohalo_$i DLA_WGRAD_DEFER=3x3 DLA_HALO_WGRAD=0 RACE_NODP=1 || exit 1
  run halo_$i DLA_WGRAD_DEFER=3x3 RACE_NODP=1 || exit 1
done
