#!/bin/bash
# GPU session: parity tests, then a bench with the per-op device-time table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-r}
timeout -k 10 900 python -m pytest tests -q -m gpu -x -rf > gpurun_out/tests_$TAG.log 2>&1 \
  && timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
       --profile-ops gpurun_out/ops_$TAG.txt > gpurun_out/bench_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
tail -2 gpurun_out/bench_$TAG.log
exit $rc
