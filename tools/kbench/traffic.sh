#!/bin/bash
# HBM traffic of one kbench op from PMC counters (MI355X_MICROARCH.md "HBM"):
# one rocprofv3 --pmc pass per counter (FETCH_SIZE costs 3 TCC counters, WRITE_SIZE 2),
# FETCH_SIZE doubled (gfx950 tallies 128-B read requests at 64 B), WRITE_SIZE as is.
#   OP=fwd|dgrad|wgrad SHAPE="N Ci H W Co k s p d" LABEL=<op label> traffic.sh TAG
# Writes gpurun_out/traffic_TAG.json: per kernel name, avg KB per dispatch of each counter,
# and the corrected bytes per launch of the op (sum over its kernels).
cd "$(dirname "$0")/_build"
OP=${OP:-wgrad}
TAG=${1:-x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SHAPE="${SHAPE:-2 20 1024 1024 16 5 2 2 1}"
REPS=${REPS:-10}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- ./kbench $OP $SHAPE $REPS \
      > $OUT/$c.log 2>&1 || { echo "pass $c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python3 - "$OUT" "$TAG" "$OP" "$SHAPE" "$REPS" "${LABEL:-}" <<'EOF'
import csv, collections, glob, json, sys
out, tag, op, shape, reps, label = sys.argv[1:7]
per = collections.defaultdict(lambda: collections.defaultdict(list))
def kname(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n[:n.index(">") + 1] if "<" in n.split("(")[0] else n.split("(")[0]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            per[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
kern = {}
total = 0.0
for k, d in per.items():
    nd = max(1, len(d.get("FETCH_SIZE", [])))
    fs = sum(d.get("FETCH_SIZE", [0])) / nd  # KB per dispatch
    ws = sum(d.get("WRITE_SIZE", [0])) / max(1, len(d.get("WRITE_SIZE", [])))
    kern[k] = {"dispatches": nd, "FETCH_SIZE_kb_per_dispatch": fs, "WRITE_SIZE_kb_per_dispatch": ws}
    if not k.startswith("__amd_rocclr"):  # the op's own kernel(s): one dispatch per launch
        total += (2.0 * fs + ws) * 1024.0
res = {"op": op, "shape": shape, "label": label, "kernels": kern,
       "hbm_bytes_per_launch": total,
       "correction": "2*FETCH_SIZE + WRITE_SIZE per dispatch (KB->B); gfx950 FETCH_SIZE halves 16-B/lane reads"}
json.dump(res, open(f"{out}/../traffic_{tag}.json", "w"), indent=1)
print(json.dumps(res))
EOF
