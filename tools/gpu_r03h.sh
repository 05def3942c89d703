set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 ISG_NO_S2K5=1
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/instancesegmentation_amd
STEPS=200 bash tools/gpu_ab.sh rep 2 "-" "ISG_LIB=$L/libisg_rep2.so ISG_STAT_REP=2 ISG_NO_BN_FINAL=1" "ISG_LIB=$L/libisg_rep4.so ISG_STAT_REP=4 ISG_NO_BN_FINAL=1" "ISG_LIB=$L/libisg_rep8.so ISG_STAT_REP=8 ISG_NO_BN_FINAL=1" "ISG_LIB=$L/libisg_rep8.so ISG_STAT_REP=8"
