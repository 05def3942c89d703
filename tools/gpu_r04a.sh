set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -rf --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/tests_r4a.log 2>&1 || { tail -30 gpurun_out/tests_r4a.log; exit 1; }
tail -1 gpurun_out/tests_r4a.log
cd tools/kbench/_build
L2="2 16 512 512 16 5 2 2 1"
for F in "ISG_NO_S2K5_WGRAD=1" "ISG_X=1" "ISG_S2W_WGS=256" "ISG_S2W_WGS=1024"; do
  echo "== $F"; env $F timeout -k 5 60 ./kbench wgrad $L2 50 | head -1 || exit 1
done
cd ../../..
STEPS=200 bash tools/gpu_ab.sh r4a 2 "ISG_NO_S2K5_WGRAD=1" "-"  || exit 1
