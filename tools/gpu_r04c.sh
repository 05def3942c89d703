set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 120 --timeout-method thread > gpurun_out/tests_r4c.log 2>&1 || { tail -30 gpurun_out/tests_r4c.log; exit 1; }
tail -1 gpurun_out/tests_r4c.log


timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 15 --profile-ops gpurun_out/ops_r4c.txt > gpurun_out/bench_r4c.log 2>&1 || { tail -30 gpurun_out/bench_r4c.log; exit 1; }
tail -1 gpurun_out/bench_r4c.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r4c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_r4c.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_prof_r4c.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_r4c -name "*stats*"
