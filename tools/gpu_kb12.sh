set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -rf --timeout 120 --timeout-method thread -k "s2k5_wgrad or wgrad_dense" > gpurun_out/tests_kb12.log 2>&1 || { tail -30 gpurun_out/tests_kb12.log; exit 1; }
tail -1 gpurun_out/tests_kb12.log
cd tools/kbench/_build || exit 1
L2="2 16 512 512 16 5 2 2 1"
for d in 0 1 2 4 3; do
  echo "== dbg=$d"; KB_STAMPS_DOWN=1 ISG_S2W_DBG=$d timeout -k 5 60 ./kbench wgrad $L2 50 || exit 1
done
echo "== 1024 WGs"; KB_STAMPS_DOWN=1 ISG_S2W_WGS=1024 timeout -k 5 60 ./kbench wgrad $L2 50 || exit 1
echo "== 256 WGs"; KB_STAMPS_DOWN=1 ISG_S2W_WGS=256 timeout -k 5 60 ./kbench wgrad $L2 50 || exit 1
