set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
ISG_BN_FUSE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_segment.py tests/test_gpu_trainer.py tests/test_gpu_blocks.py tests/test_gpu_kp_stem.py tests/test_gpu_infer.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_fuse.log 2>&1; rc=$?; tail -3 gpurun_out/t_fuse.log; [ $rc -ne 0 ] && exit $rc
tools/gpu_ab.sh fuse 2 "-" "ISG_BN_FUSE=1"
