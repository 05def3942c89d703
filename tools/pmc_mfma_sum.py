"""Per-kernel summary of tools/pmc_mfma.sh's counter pass (rocprofv3 counter_collection.csv)."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(f"{out}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:58]
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES":
            cnt[n] += 1
rows = sorted(acc.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))
lines = ["kernel                                                      disp  kcyc/disp  mfma%  "
         "wait_any% wait_inst% active%  valu/wave"]
for n, d in rows[:45]:
    disp = max(cnt[n], 1)
    kcyc = d.get("GRBM_GUI_ACTIVE", 0) / 8.0  # the 8 XCDs' cycles summed
    wc = max(d.get("SQ_WAVE_CYCLES", 0), 1)
    wv = max(d.get("SQ_WAVES", 0), 1)
    mf = 100.0 * d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(kcyc * 1024, 1)
    lines.append(f"{n:58s} {disp:5d} {kcyc / disp:10.0f} {mf:6.1f} {100 * d.get('SQ_WAIT_ANY', 0) / wc:9.1f} "
                 f"{100 * d.get('SQ_WAIT_INST_ANY', 0) / wc:10.1f} {100 * d.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.1f} "
                 f"{d.get('SQ_INSTS_VALU', 0) / wv:10.0f}")
open(f"{out}/summary.txt", "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
