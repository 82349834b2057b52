#!/bin/bash
# Round 3, call 11: (1) why the fp32 GoogLeNet CLI step took ~1 s (MIOpen immediate mode vs MIOpen off,
# torch.profiler top ops); (2) eager virtual-rank ring timing with the ring search cached (g08b's eager
# rows paid a 3.5 ms Python ring search per call whenever channels > 1).
set -o pipefail
O=gpurun_out/g11; mkdir -p $O
timeout -k 10 240 python -u scripts/runs/probes/fp32_googlenet_probe.py --configs immediate,nomiopen --profile immediate > $O/fp32_probe.log 2>&1 || { tail -40 $O/fp32_probe.log; exit 1; }
grep '^{' $O/fp32_probe.log
timeout -k 10 200 python -u scripts/vrank_ring_timing.py --out $O/vrank_eager.jsonl > $O/vrank_eager.log 2>&1 || { tail -20 $O/vrank_eager.log; exit 1; }
python scripts/fit_ring_alpha.py $O/vrank_eager.jsonl
