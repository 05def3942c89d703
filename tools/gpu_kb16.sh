set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -rf --timeout 120 --timeout-method thread -k "s2k5_wgrad or wgrad_dense" > gpurun_out/tests_kb16.log 2>&1 || { tail -30 gpurun_out/tests_kb16.log; exit 1; }
tail -1 gpurun_out/tests_kb16.log
cd tools/kbench/_build || exit 1
L2="2 16 512 512 16 5 2 2 1"
for F in "ISG_X=1" "ISG_S2W_DBG=2" "ISG_S2W_DBG=4"; do
  echo "== $F"; env KB_STAMPS_DOWN=1 $F timeout -k 5 60 ./kbench wgrad $L2 50 || exit 1
done
cd $GRAFT_REPO_ROOT
STEPS=200 bash tools/gpu_ab.sh kb16 2 "ISG_NO_S2K5_WGRAD=1" "-"  || exit 1
