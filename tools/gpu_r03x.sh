set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
STEPS=200 bash tools/gpu_ab.sh r3x 2 "-" "ISG_PWG_TPB=1" "ISG_PWG_TPB=3" "ISG_SIDE_BATCH=12" "ISG_SIDE_BATCH=48" "ISG_PWX_MINB=384" "ISG_PWX_MINB=768" || exit 1
