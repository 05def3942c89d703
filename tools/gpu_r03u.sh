set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
STEPS=200 bash tools/gpu_ab.sh r3u 3 "-" "ISG_BN_FINAL_COUNT=1099511627776" || exit 1
