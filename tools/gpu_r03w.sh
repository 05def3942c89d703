set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 120 --timeout-method thread > gpurun_out/tests_r3w.log 2>&1 || { tail -30 gpurun_out/tests_r3w.log; exit 1; }
tail -1 gpurun_out/tests_r3w.log
bash tools/gpu_ktrace.sh r3w "ISG_DUMMY=0"
