#!/bin/bash
# full GPU parity suite, then the default step timed in 3 runs of 100 steps
cd $GRAFT_REPO_ROOT && export PYTHONDONTWRITEBYTECODE=1 && mkdir -p gpurun_out
TAG=${1:-full}
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x -rf --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/tests_$TAG.log | tail -20; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
AB="${AB:--}" bash tools/gpu_ab2.sh $TAG 3
