#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
run() {
  echo "=== $*" >> gpurun_out/dbg.log
  env "$@" >> gpurun_out/dbg.log 2>&1
  rc=$?
  echo "rc=$rc" >> gpurun_out/dbg.log
  if [ $rc -gt 1 ]; then exit $rc; fi
}
run ISG_GENERIC_CONV=1 timeout -k 10 300 python -m pytest tests/test_gpu_blocks.py -q -m gpu -rf
run ISG_GENERIC_CONV=1 ISG_DEBUG_POISON=1 timeout -k 10 300 python -m pytest tests/test_gpu_segment.py -q -m gpu -rf -s -k segment3
run X=1 timeout -k 10 300 python -m pytest tests/test_gpu_segment.py -q -m gpu -rf -s
grep -E "===|rc=|worst|passed|failed" gpurun_out/dbg.log
