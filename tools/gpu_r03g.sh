set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="tests/test_gpu_trainer.py::test_trainer_full_size_step_matches_oracle"
for e in "ISG_GRAD_PROFILE=1" "ISG_NO_HEAD=1" "ISG_SUB2_DIRECT=1" "ISG_NO_S2K5=1"; do
  env $e timeout -k 10 300 python -u -m pytest "$T" -x -q -m gpu -s --timeout 200 --timeout-method thread -k 1344 > gpurun_out/t1344_${e%%=*}.log 2>&1
  echo "$e rc=$? $(grep -o 'worst.*' gpurun_out/t1344_${e%%=*}.log | cut -c1-300)"
done
STEPS=200 bash tools/gpu_ab.sh bnf 1 "-" "ISG_BN_FUSE=1" "ISG_NO_BN_FINAL=1"
L=$GRAFT_REPO_ROOT/instancesegmentation_amd
STEPS=200 bash tools/gpu_ab.sh rep 1 "ISG_LIB=$L/libisg_rep4.so ISG_STAT_REP=4" "ISG_LIB=$L/libisg_rep4.so ISG_STAT_REP=4 ISG_NO_BN_FINAL=1" "ISG_LIB=$L/libisg_rep1.so ISG_STAT_REP=1 ISG_NO_BN_FINAL=1" "ISG_LIB=$L/libisg_rep4.so ISG_STAT_REP=4 ISG_BN_FUSE=1"
