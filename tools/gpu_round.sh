#!/bin/bash
# GPU session: parity tests -> smoke -> bench (+ per-op table) -> rocprofv3 kernel-trace stats of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-r}
STEPS=${STEPS:-20}
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -rf --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 5 --cpu-seconds 15 \
    --profile-ops gpurun_out/ops_$TAG.txt > gpurun_out/bench_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -2 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 5 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*stats*"
