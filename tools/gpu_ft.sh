#!/bin/bash
# round-6: fused step tail parity (trainer + DP tests), then interleaved A/B of the step
cd $GRAFT_REPO_ROOT && export PYTHONDONTWRITEBYTECODE=1 && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_dp.py -v -x --timeout 120 \
    --timeout-method thread -m gpu > gpurun_out/tests_ft.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/tests_ft.log | tail -25
[ $rc -eq 0 ] || exit 1
B="ISG_SIDE_BATCH=16 ISG_FORK_DELAY=0"
AB="-;ISG_NO_FUSED_TAIL=1;ISG_MAX_INFLIGHT=1;ISG_NO_DW_FUSE=1;ISG_NO_DW_FUSE=1 ISG_MAX_INFLIGHT=1;$B # --eager;$B ISG_NO_DW_FUSE=1 # --eager" \
    bash tools/gpu_ab2.sh ft 3
