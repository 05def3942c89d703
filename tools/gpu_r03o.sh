set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 120 --timeout-method thread > gpurun_out/tests_r3o.log 2>&1 || { tail -30 gpurun_out/tests_r3o.log; exit 1; }
tail -1 gpurun_out/tests_r3o.log
L=$GRAFT_REPO_ROOT/instancesegmentation_amd
STEPS=200 bash tools/gpu_ab.sh r3o 3 "ISG_LIB=$L/libisg_prev.so" "-" || exit 1
cd tools/kbench/_build || exit 1
for S in "fwd 2 128 64 64 48 1 1 0 1" "dgrad 2 48 64 64 128 1 1 0 1"; do
  echo "== $S stats"; timeout -k 5 60 ./kbench $S 100
done
