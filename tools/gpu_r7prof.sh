#!/bin/bash
# Round-5 measurement: bench line (default flags) + a rocprofv3 kernel-trace of the training
# leg ALONE (--dominant skips the per-op pass; no infer / dense / dp legs), so the kernel
# stats come from training steps at the bench shape only and the roofline op's average
# duration can be compared with the bench line's stamp-timed value.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-r7}
DOM=${DOM:-bwd:d_out0}
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 15 \
    --profile-ops gpurun_out/ops_$TAG.txt > gpurun_out/bench_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
    --no-dense-leg --no-dp-leg --dominant $DOM \
    > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*stats*"
