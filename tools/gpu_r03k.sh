set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 120 --timeout-method thread > gpurun_out/tests_r3k.log 2>&1 || { tail -30 gpurun_out/tests_r3k.log; exit 1; }
tail -1 gpurun_out/tests_r3k.log
STEPS=200 bash tools/gpu_ab.sh fincnt 2 "-" "ISG_BN_FINAL_COUNT=1099511627776" "ISG_BN_FINAL_COUNT=32768" || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer --no-dense-leg --profile-ops gpurun_out/ops_r3k.txt > gpurun_out/bench_r3k.log 2>&1; tail -1 gpurun_out/bench_r3k.log | cut -c1-300
# kbench: finalised BN coefficients (KB_COEF=1) vs consumer-side evaluation from the
# statistics, on the op shapes that carry most of the step
set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build || exit 1
for S in "dgrad 2 128 64 64 48 1 1 0 1" "dgrad 2 48 64 64 128 1 1 0 1" "fwd 2 128 64 64 48 1 1 0 1" \
         "fwd 2 48 64 64 128 1 1 0 1" "fwd 2 4 256 256 16 1 1 0 1" "fwd 2 16 256 256 4 1 1 0 1" \
         "wgrad 2 48 64 64 128 1 1 0 1" "wgrad 2 128 64 64 48 1 1 0 1" "dgrad 2 16 128 128 48 1 1 0 1"; do
  a=$(KB_COEF=1 timeout -k 5 60 ./kbench $S 100 | head -1); b=$(timeout -k 5 60 ./kbench $S 100 | head -1)
  echo "$S | coef: $a | stats: $b"
done
