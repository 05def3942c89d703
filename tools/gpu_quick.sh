#!/bin/bash
# quick GPU iteration: parity tests + bench with per-op table (no CPU baseline, no profiler)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-q}
K=${2:-}
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -rf --timeout 120 --timeout-method thread $K \
    > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/tests_$TAG.log | tail -30; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --profile-ops gpurun_out/ops_$TAG.txt > gpurun_out/bench_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
