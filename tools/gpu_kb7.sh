# kbench stamps of the slab 1x1 kernel after exact per-lane load counts
set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build || exit 1
for S in "fwd 2 128 64 64 48 1 1 0 1" "dgrad 2 48 64 64 128 1 1 0 1" "fwd 2 48 128 128 16 1 1 0 1"; do
  echo "== $S coef"; KB_COEF=1 timeout -k 5 60 ./kbench $S 100
  echo "== $S stats"; timeout -k 5 60 ./kbench $S 100
done
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_blocks.py tests/test_gpu_segment.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_kb7.log 2>&1 || { tail -30 gpurun_out/t_kb7.log; exit 1; }
tail -1 gpurun_out/t_kb7.log
STEPS=200 bash tools/gpu_ab.sh kb7 1 "-"
# kbench: the M=128 / K=48 1x1 GEMMs at 64^2 (pw_kernel<2> today) on the slab kernel
# under explicit (BM, BP) tiles
set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build || exit 1
for S in "fwd 2 48 64 64 128 1 1 0 1" "dgrad 2 128 64 64 48 1 1 0 1"; do
  echo "$S default: $(timeout -k 5 60 ./kbench $S 100 | head -1 | cut -d: -f2)"
  for T in "128 16" "64 32" "32 64" "64 64"; do
    set -- $T
    echo "$S slab BM=$1 BP=$2: $(ISG_PW_SLAB_ALL=1 ISG_PWX_BM=$1 ISG_PWX_BP=$2 timeout -k 5 60 ./kbench $S 100 | head -1 | cut -d: -f2)"
  done
done
