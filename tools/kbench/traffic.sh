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
python3 - "$OUT" "$TAG" "$OP" "$SHAPE" "$REPS" "${LABEL:-}" "${CONFIG:-}" <<'EOF'
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
# Dominant global-load width per kernel (bytes per lane). MI355X_MICROARCH.md (HBM): gfx950
# FETCH_SIZE reports exactly half the bytes of 16-B/lane streaming reads; other widths are
# uncalibrated — those kernels' FETCH_SIZE is reported as read, not doubled.
LOAD_WIDTH = {"pwx_kernel": 16, "thin_pw_kernel": 16, "sub2_dgrad_lds_kernel": 16,
              "s2k5_fwd_kernel": 16, "down_conv_kernel": 16, "down_wgrad_kernel": 16,
              "tap_conv_kernel": 8, "sub2_dgrad_mfma_kernel": 4, "pw_kernel": 4,
              "head_fwd_kernel": 4, "head_bwd_kernel": 4, "tap_wgrad_kernel": 8,
              "tap_wgrad_all_kernel": 8}
def width(k):
    for p, w in LOAD_WIDTH.items():
        if k.startswith(p):
            return w
    return 0
kern = {}
total = 0.0
for k, d in per.items():
    nd = max(1, len(d.get("FETCH_SIZE", [])))
    fs = sum(d.get("FETCH_SIZE", [0])) / nd  # KB per dispatch
    ws = sum(d.get("WRITE_SIZE", [0])) / max(1, len(d.get("WRITE_SIZE", [])))
    w = width(k)
    scale = 2.0 if w == 16 else 1.0
    kern[k] = {"dispatches": nd, "FETCH_SIZE_kb_per_dispatch": fs, "WRITE_SIZE_kb_per_dispatch": ws,
               "load_bytes_per_lane": w or None, "fetch_scale": scale}
    if not k.startswith("__amd_rocclr"):  # the op's own kernel(s): one dispatch per launch
        total += (scale * fs + ws) * 1024.0
res = {"op": op, "shape": shape, "label": label, "kernels": kern,
       "hbm_bytes_per_launch": total,
       "correction": "fetch_scale*FETCH_SIZE + WRITE_SIZE per dispatch (KB->B); fetch_scale 2 only "
                     "for 16-B/lane streaming loads (gfx950 FETCH_SIZE halves those), 1 "
                     "(uncalibrated) for narrower loads"}
if len(sys.argv) > 7 and sys.argv[7]:
    res["config"] = [int(v) for v in sys.argv[7].split(",")]
json.dump(res, open(f"{out}/../traffic_{tag}.json", "w"), indent=1)
print(json.dumps(res))
EOF
