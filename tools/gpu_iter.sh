#!/bin/bash
# One GPU iteration: selected parity tests, then kbench lines.
#   K="pytest -k expr" KB="op shape...;op shape..." KENV="VAR=val ..." tools/gpu_iter.sh TAG
# -> gpurun_out/it_TAG_tests.log, gpurun_out/it_TAG_kb.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-x}
if [ -n "${K:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -v -m gpu -x -rf --timeout 300 --timeout-method thread -k "$K" \
      > gpurun_out/it_${TAG}_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/it_${TAG}_tests.log | tail -40; exit 1; }
  tail -2 gpurun_out/it_${TAG}_tests.log
fi
if [ -n "${KB:-}" ]; then
  IFS=';' read -ra LINES <<< "$KB"
  for l in "${LINES[@]}"; do
    env ${KENV:-} timeout -k 10 60 tools/kbench/_build/kbench $l >> gpurun_out/it_${TAG}_kb.log 2>&1 || { tail -5 gpurun_out/it_${TAG}_kb.log; exit 1; }
  done
  cat gpurun_out/it_${TAG}_kb.log
fi
