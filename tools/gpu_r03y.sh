set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
STEPS=200 bash tools/gpu_ab.sh r3y 2 "ISG_SIDE_BATCH=24" "ISG_SIDE_BATCH=36" "ISG_SIDE_BATCH=48" "ISG_SIDE_BATCH=64" "ISG_SIDE_BATCH=96" || exit 1
