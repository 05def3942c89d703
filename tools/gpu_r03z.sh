set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 120 --timeout-method thread > gpurun_out/tests_r3z.log 2>&1 || { tail -30 gpurun_out/tests_r3z.log; exit 1; }
tail -1 gpurun_out/tests_r3z.log
L=$GRAFT_REPO_ROOT/instancesegmentation_amd
STEPS=200 bash tools/gpu_ab.sh r3z 3 "ISG_NO_LATE_FORK=1" "-"  || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer --no-dense-leg --profile-ops gpurun_out/ops_r3z.txt > gpurun_out/bench_r3z.log 2>&1; tail -1 gpurun_out/bench_r3z.log | cut -c1-200
