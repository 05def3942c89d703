set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 120 --timeout-method thread > gpurun_out/tests_r4b.log 2>&1 || { tail -30 gpurun_out/tests_r4b.log; exit 1; }
tail -1 gpurun_out/tests_r4b.log
cd tools/kbench/_build || exit 1
echo "== dgrad L2"; timeout -k 5 60 ./kbench dgrad 2 16 512 512 16 5 2 2 1 50 | head -1 || exit 1
for S in "2 48 64 64 128 1 1 0 1" "2 128 64 64 48 1 1 0 1" "2 256 64 64 128 1 1 0 1" "2 16 128 128 48 1 1 0 1" "2 48 128 128 16 1 1 0 1"; do
  echo "== wgrad $S"; timeout -k 5 60 ./kbench wgrad $S 100 | head -1 || exit 1
done
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/instancesegmentation_amd
STEPS=200 bash tools/gpu_ab.sh r4b 2 "ISG_LIB=$L/libisg_prev.so" "-"  || exit 1
