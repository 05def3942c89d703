#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/d1 gpurun_out/d2 gpurun_out/d3
T="tests/test_gpu_segment.py -q -m gpu -rf -s -k train_step"
ISG_DUMP_DIR=gpurun_out/d1 ISG_GENERIC_CONV=1 timeout -k 10 300 python -m pytest $T > gpurun_out/dd1.log 2>&1
ISG_DUMP_DIR=gpurun_out/d2 ISG_GENERIC_CONV=1 timeout -k 10 300 python -m pytest $T > gpurun_out/dd2.log 2>&1
ISG_DUMP_DIR=gpurun_out/d3 timeout -k 10 300 python -m pytest $T > gpurun_out/dd3.log 2>&1
grep -h "worst\|passed\|failed" gpurun_out/dd*.log
