#!/bin/bash
# pipelined ring: virtual-rank GPU tests + timing vs the plain ring at N=8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine_vranks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2m_vranks.log 2>&1 || { echo "vrank tests failed"; tail -40 gpurun_out/r2m_vranks.log; exit 1; }
tail -1 gpurun_out/r2m_vranks.log
timeout -k 10 200 python scripts/vrank_ring_timing.py --world 8 --channels 7 --out gpurun_out/vrank_ring_pipe_timing.jsonl > gpurun_out/r2m_timing.log 2>&1 && cat gpurun_out/r2m_timing.log
timeout -k 10 200 python scripts/vrank_ring_timing.py --world 8 --channels 1 --out gpurun_out/vrank_ring_pipe_timing_c1.jsonl > gpurun_out/r2m_timing1.log 2>&1 && cat gpurun_out/r2m_timing1.log
