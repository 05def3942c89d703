set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_dp.py tests/test_gpu_kp_stem.py -q -m gpu -x -rf --timeout 120 --timeout-method thread > gpurun_out/tests_r3n.log 2>&1 || { tail -30 gpurun_out/tests_r3n.log; exit 1; }
tail -1 gpurun_out/tests_r3n.log
STEPS=200 bash tools/gpu_ab.sh r3n 3 "ISG_BUCKETS=2 ISG_NO_SIDE2=1" "ISG_NO_SIDE2=1" "-" || exit 1
