set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "dense" > gpurun_out/t_k.log 2>&1; rc=$?; tail -2 gpurun_out/t_k.log; [ $rc -ne 0 ] && exit $rc
cd tools/kbench/_build
export KB_COEF=1
for S in "2 48 128 128 16 1 1 0 1" "2 16 128 128 48 1 1 0 1" "2 128 64 64 48 1 1 0 1"; do
  for op in fwd dgrad; do timeout -k 5 60 ./kbench $op $S 50 | head -4; done
done
cd $GRAFT_REPO_ROOT
tools/gpu_ab.sh r3d 3 "-"
