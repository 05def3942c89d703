set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mask_head.py tests/test_gpu_infer.py -x -q -m gpu --timeout 120 --timeout-method thread -s > gpurun_out/t_head.log 2>&1; rc=$?; tail -12 gpurun_out/t_head.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -5 gpurun_out/t_all.log; [ $rc -ne 0 ] && exit $rc
ISG_BN_FUSE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_segment.py tests/test_gpu_trainer.py tests/test_gpu_blocks.py tests/test_gpu_kp_stem.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_fuse.log 2>&1; rc=$?; tail -3 gpurun_out/t_fuse.log; [ $rc -ne 0 ] && exit $rc
tools/gpu_ab.sh r3a 2 "-" "ISG_BN_FUSE=1" "ISG_NO_HEAD=1" "ISG_SUB2_DIRECT=1"
