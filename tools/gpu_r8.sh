#!/bin/bash
# Round-6 GPU session: parity tests -> smoke -> bench line (+ per-op table) -> host floors of
# graph replay and of the eager C++ executor -> rocprofv3 kernel trace of the training leg
# alone (the roofline op's rocprof average against the line's stamps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-r8}
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -rf --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
fi
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 15 \
    --profile-ops gpurun_out/ops_$TAG.txt > gpurun_out/bench_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 200 python -u tools/replay_host.py --steps 100 > gpurun_out/rh_graph_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/rh_graph_$TAG.log; exit 1; }
timeout -k 10 200 python -u tools/replay_host.py --steps 100 --eager > gpurun_out/rh_eager_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/rh_eager_$TAG.log; exit 1; }
cat gpurun_out/rh_graph_$TAG.log gpurun_out/rh_eager_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
    --no-dense-leg --no-dp-leg --dominant ${DOM:-bwd:d_out0} \
    > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*stats*"
