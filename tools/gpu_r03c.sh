set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
tools/gpu_ab.sh r3c 2 "-" "ISG_NO_HEAD=1" "ISG_NO_S2K5=1" "ISG_SUB2_DIRECT=1"
STEPS=20 tools/gpu_ktrace.sh r3c "ISG_DUMMY=0"
