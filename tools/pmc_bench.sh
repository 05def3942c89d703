#!/bin/bash
# HBM traffic of the bench's dominant kernel from PMC counters (MI355X_MICROARCH.md "HBM"):
# one rocprofv3 --pmc pass per counter over a short bench run, the kernel picked by name.
#   KERNEL=<kernel name prefix> LABEL=<op label> [GRID=<threads>] [PER=n NTH=i] pmc_bench.sh TAG
# GRID keeps dispatches of that grid size; PER/NTH keep the i-th of every n matching
# dispatches (a kernel two ops of a step share, e.g. both stem weight gradients).
# FETCH_SIZE doubled (gfx950 tallies 128-B read requests at 64 B), WRITE_SIZE as is; writes
# gpurun_out/traffic_TAG.json with the corrected bytes per dispatch of that kernel.
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
OUT=$GRAFT_REPO_ROOT/gpurun_out/traffic_$TAG
mkdir -p $OUT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-roofline --no-cpu-baseline \
      --no-infer --no-dense-leg > $OUT/$c.log 2>&1) || { echo "pass $c failed"; tail -5 $OUT/$c.log; exit 1; }
done
python3 - "$OUT" "$TAG" "${KERNEL:?}" "${LABEL:?}" "${GRID:-0}" "${PER:-1}" "${NTH:-0}" <<'PY'
import csv, glob, json, sys
out, tag, kernel, label = sys.argv[1:5]
grid, per, nth = (int(v) for v in sys.argv[5:8])
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
for c in vals:
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        rows = []
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            if n.startswith(kernel) and r["Counter_Name"] == c and \
                    (grid == 0 or int(r["Grid_Size"]) == grid):
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        rows.sort()
        vals[c] += [v for i, (_, v) in enumerate(rows) if i % per == nth]
fs = sum(vals["FETCH_SIZE"]) / max(1, len(vals["FETCH_SIZE"]))
ws = sum(vals["WRITE_SIZE"]) / max(1, len(vals["WRITE_SIZE"]))
res = {"op": "bench", "label": label, "config": [2, 20, 1024],
       "shape": "bench.py --steps 3 --warmup 1 (bs2 1024^2, keypoint input)",
       "kernels": {kernel: {"dispatches": len(vals["FETCH_SIZE"]), "FETCH_SIZE_kb_per_dispatch": fs,
                            "WRITE_SIZE_kb_per_dispatch": ws}},
       "hbm_bytes_per_launch": (2.0 * fs + ws) * 1024.0,
       "correction": "2*FETCH_SIZE + WRITE_SIZE per dispatch (KB->B); gfx950 FETCH_SIZE halves 16-B/lane reads"}
json.dump(res, open(f"{out}/../traffic_{tag}.json", "w"), indent=1)
print(json.dumps(res))
PY
