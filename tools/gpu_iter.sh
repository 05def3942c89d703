#!/bin/bash
# One build-measure iteration on the GPU box: parity tests (pytest -k filter in $1, "" =
# all GPU tests), then the bench with the per-op device-time table. Tag in $2.
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
K=${1:-}
TAG=${2:-it}
if [ -n "$K" ]; then KF=(-k "$K"); else KF=(); fi
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread "${KF[@]}" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
    --profile-ops gpurun_out/ops_$TAG.txt > gpurun_out/bench_$TAG.log 2>&1
rc=$?
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
exit $rc
