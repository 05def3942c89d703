set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mask_head.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "dense or head" > gpurun_out/t_k.log 2>&1; rc=$?; tail -3 gpurun_out/t_k.log; [ $rc -ne 0 ] && exit $rc
cd tools/kbench/_build
export KB_COEF=1
S="2 16 512 512 16 5 2 2 1"
timeout -k 5 60 ./kbench fwd $S 50 && timeout -k 5 60 ./kbench dgrad $S 50
H="2 16 256 256 16 1 1 0 1"
timeout -k 5 60 ./kbench headf $H 50 && timeout -k 5 60 ./kbench headb $H 50
cd $GRAFT_REPO_ROOT
OP=fwd SHAPE="$S" FILTER=s2k5 timeout -k 5 200 bash tools/kbench/pmc.sh s2k5b
OP=headb SHAPE="$H" FILTER=head_bwd timeout -k 5 200 bash tools/kbench/pmc.sh headbb
