#!/bin/bash
set -o pipefail
O=gpurun_out/g28; mkdir -p $O
timeout -k 10 120 python3 scripts/stream_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep "^M=" $O/probe.log
