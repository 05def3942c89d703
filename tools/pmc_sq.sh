#!/bin/bash
# SQ counters (wave cycles split into active / waiting) per kernel over a short bench run:
# one rocprofv3 --pmc pass (8 SQ counters), gpurun_out/pmc_sq_TAG/ + a per-kernel summary.
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d $OUT -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-roofline --no-cpu-baseline \
    --no-infer --no-dense-leg > $OUT/run.log 2>&1) || { echo "pmc pass failed"; tail -5 $OUT/run.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(f"{out}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:60]
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            cnt[n] += 1
rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
with open(f"{out}/summary.txt", "w") as fo:
    fo.write("kernel dispatches waves wave_cyc wait_any% wait_inst% active% valu/wave vmem/wave\n")
    for n, d in rows[:40]:
        wc = max(d.get("SQ_WAVE_CYCLES", 0), 1)
        wv = max(d.get("SQ_WAVES", 0), 1)
        fo.write(f"{n:60s} {cnt[n]:5d} {wv:9.0f} {wc:12.0f} {100*d.get('SQ_WAIT_ANY',0)/wc:6.1f} "
                 f"{100*d.get('SQ_WAIT_INST_ANY',0)/wc:6.1f} {100*d.get('SQ_ACTIVE_INST_ANY',0)/wc:6.1f} "
                 f"{d.get('SQ_INSTS_VALU',0)/wv:8.0f} {d.get('SQ_INSTS_VMEM_RD',0)/wv:6.0f}\n")
print(open(f"{out}/summary.txt").read())
PY
