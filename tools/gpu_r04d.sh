set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 15 --profile-ops gpurun_out/ops_r4d.txt > gpurun_out/bench_r4d.log 2>&1 || { tail -30 gpurun_out/bench_r4d.log; exit 1; }
tail -1 gpurun_out/bench_r4d.log | cut -c1-200
