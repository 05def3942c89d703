#!/bin/bash
# keypoint-stem parity tests, then the bench (keypoint + dense legs, per-op table)
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-kp}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kp_stem.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|err |logits" gpurun_out/tests_$TAG.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
    --profile-ops gpurun_out/ops_$TAG.txt > gpurun_out/bench_$TAG.log 2>&1
rc=$?
tail -1 gpurun_out/bench_$TAG.log | cut -c1-1500
exit $rc
