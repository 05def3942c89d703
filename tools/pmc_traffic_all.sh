#!/bin/bash
# HBM-side bytes per dispatch for every kernel of a short bench run: two rocprofv3 --pmc
# passes (FETCH_SIZE, WRITE_SIZE), FETCH_SIZE doubled (gfx950 tallies 128-B read requests
# at 64 B, MI355X_MICROARCH.md "HBM"). -> gpurun_out/traffic_all_TAG/summary.txt
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic_all_$TAG
mkdir -p $OUT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-roofline --no-cpu-baseline \
      --no-infer --no-dense-leg > $OUT/$c.log 2>&1) || { echo "pass $c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_traffic_sum.py $OUT
