set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_kp_stem.py -x -q -m gpu --timeout 120 --timeout-method thread -k "dense or kp" > gpurun_out/t_k.log 2>&1; rc=$?; tail -2 gpurun_out/t_k.log; [ $rc -ne 0 ] && exit $rc
(cd tools/kbench/_build && KB_COEF=1 timeout -k 5 60 ./kbench fwd 2 16 512 512 16 5 2 2 1 50)
tools/gpu_ab.sh r3c 2 "-" "ISG_NO_HEAD=1" "ISG_NO_S2K5=1" "ISG_SUB2_DIRECT=1"
STEPS=20 tools/gpu_ktrace.sh r3c "ISG_DUMMY=0"
