"""Per-kernel HBM bytes per dispatch from tools/pmc_traffic_all.sh's two counter passes:
FETCH_SIZE (x2, the gfx950 correction) and WRITE_SIZE, both in KB per dispatch."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
acc = {c: collections.defaultdict(list) for c in ("FETCH_SIZE", "WRITE_SIZE")}
for c in acc:
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != c:
                continue
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:58]
            acc[c][n].append(float(r["Counter_Value"]) * 1024)  # KB -> B
names = sorted(acc["FETCH_SIZE"], key=lambda n: -sum(acc["FETCH_SIZE"][n]))
lines = ["kernel                                                      disp  read MB/disp  write MB/disp"]
for n in names[:45]:
    fe = acc["FETCH_SIZE"][n]
    wr = acc["WRITE_SIZE"].get(n, [0.0])
    lines.append(f"{n:58s} {len(fe):5d} {2 * sum(fe) / len(fe) / 1e6:13.3f} {sum(wr) / len(wr) / 1e6:14.3f}")
open(f"{out}/summary.txt", "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
