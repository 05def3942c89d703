set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
STEPS=20 tools/gpu_envcmp.sh r3b "ISG_DUMMY=0" "ISG_NO_HEAD=1 ISG_SUB2_DIRECT=1 ISG_NO_S2K5=1"
