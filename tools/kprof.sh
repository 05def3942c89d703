#!/bin/bash
# rocprofv3 kernel traces of single kbench lines: GPU-side kernel durations (no host launch
# overhead). KB="op shape...;..." [KENV="VAR=val"] tools/kprof.sh TAG
# -> gpurun_out/kprof_TAG/<i>/kp_results.db, summary printed (tools/kprof_sum.py)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-x}
IFS=';' read -ra LINES <<< "$KB"
i=0
for l in "${LINES[@]}"; do
  i=$((i+1))
  env ${KENV:-} timeout -k 10 90 rocprofv3 --kernel-trace -d gpurun_out/kprof_$TAG/$i -o kp -- tools/kbench/_build/kbench $l > gpurun_out/kprof_${TAG}_$i.log 2>&1 || { tail -5 gpurun_out/kprof_${TAG}_$i.log; exit 1; }
  echo "== [${KENV:-}] $l"
  python3 tools/kprof_sum.py gpurun_out/kprof_$TAG/$i/kp_results.db || exit 1
done
