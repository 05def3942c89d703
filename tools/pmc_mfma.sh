#!/bin/bash
# MFMA utilisation and wave-cycle split per kernel over a short bench run: one rocprofv3
# --pmc pass (7 SQ counters + GRBM_GUI_ACTIVE), gpurun_out/pmc_mfma_TAG/ + a summary.
#   mfma% = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
#   (16x16x4 f32 MFMA: 32 busy cycles per SIMD each; GUI_ACTIVE sums the 8 XCDs' cycles)
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_mfma_$TAG
mkdir -p $OUT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv \
    -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-roofline \
    --no-cpu-baseline --no-infer --no-dense-leg > $OUT/run.log 2>&1) || { echo "pmc pass failed"; tail -5 $OUT/run.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/pmc_mfma_sum.py $OUT
