#!/bin/bash
# trainer/DP parity tests, then a rocprofv3 kernel trace of the default bench step
cd $GRAFT_REPO_ROOT && export PYTHONDONTWRITEBYTECODE=1 && mkdir -p gpurun_out
TAG=${1:-tr}
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_dp.py -v -x --timeout 120 \
    --timeout-method thread -m gpu > gpurun_out/tests_$TAG.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" gpurun_out/tests_$TAG.log | tail -5
[ $rc -eq 0 ] || exit 1
bash tools/gpu_trace_env.sh $TAG
