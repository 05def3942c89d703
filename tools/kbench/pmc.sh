#!/bin/bash
# PMC passes over one kbench shape (one counter group per run, per MI355X_MICROARCH.md)
#   OP=fwd|dgrad|wgrad SHAPE="N Ci H W Co k s p d" FILTER=<kernel-name substring> pmc.sh TAG
cd "$(dirname "$0")/_build"
OP=${OP:-wgrad}
FILTER=${FILTER:-wgrad}
TAG=${1:-x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SHAPE="${SHAPE:-2 128 64 64 48 1 1 0 1}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- ./kbench $OP $SHAPE 10 > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
for f in $(find $OUT -name "*counter_collection.csv"); do python3 -c "
import csv,sys,collections
agg=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open('$f')):
    if '$FILTER' in r['Kernel_Name']:
        agg[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
for k in agg: print('%-24s %14.0f' % (k, agg[k]/max(1,n[k])))
"; done
