#!/bin/bash
# Host cost of a step (graph replay vs the eager C++ executor, idle-queue issue) and a
# rocprofv3 kernel trace of the EAGER step (bench --eager), to compare its timeline with
# the graph's (tools/step_timeline.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-e}
timeout -k 10 200 python -u tools/replay_host.py --steps 100 > gpurun_out/rh_graph_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/rh_graph_$TAG.log; exit 1; }
timeout -k 10 200 python -u tools/replay_host.py --steps 100 --eager > gpurun_out/rh_eager_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/rh_eager_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rh_graph_$TAG.log gpurun_out/rh_eager_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/kte_$TAG -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
    --no-dense-leg --no-dp-leg --no-roofline --eager \
    > $GRAFT_REPO_ROOT/gpurun_out/bench_kte_$TAG.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_kte_$TAG.log; exit 1; }
grep "^{" $GRAFT_REPO_ROOT/gpurun_out/bench_kte_$TAG.log | cut -c1-300
