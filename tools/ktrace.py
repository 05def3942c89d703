"""Timeline analysis of a rocprofv3 kernel trace of bench.py (tools/gpu_ktrace.sh).

  python tools/ktrace.py gpurun_out/kt_TAG_0 [gpurun_out/kt_TAG_1 ...]

Per run: the timed steps' wall time, the GPU-busy union, the time two or more kernels
overlap, and the in-graph per-kernel-name totals per step (top 25); with two runs, the
per-kernel-name per-step difference."""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def analyse(d, nsteps_hint=20):
    rows = load(d)
    # the timed region: the last `nsteps_hint` occurrences of the Adam kernel mark steps
    adam = [i for i, r in enumerate(rows) if "adam" in r[2].lower()]
    if len(adam) > nsteps_hint:
        first = adam[-nsteps_hint - 1] + 1
        rows = rows[first:adam[-1] + 1]
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    busy = over = 0
    cur_s = cur_e = None
    ev = sorted([(s, 1) for s, _, _ in rows] + [(e, -1) for _, e, _ in rows])
    depth, last = 0, t0
    for t, d_ in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            over += t - last
        depth += d_
        last = t
    per = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in rows:
        k = n.replace("void ", "").replace("(anonymous namespace)::", "")
        k = k.split("(")[0].strip()
        per[k] += (e - s) / 1e3
        cnt[k] += 1
    steps = nsteps_hint
    print(f"{d}: wall {(t1 - t0) / 1e3 / steps:.1f} us/step, busy {busy / 1e3 / steps:.1f}, "
          f"overlap>=2 {over / 1e3 / steps:.1f}, kernel sum {sum(per.values()) / steps:.1f}, "
          f"kernels/step {len(rows) / steps:.0f}")
    return {k: v / steps for k, v in per.items()}, {k: c / steps for k, c in cnt.items()}


def main():
    ds = sys.argv[1:]
    res = [analyse(d) for d in ds]
    top = sorted(res[0][0].items(), key=lambda kv: -kv[1])[:25]
    for k, v in top:
        line = f"  {v:8.1f} us/step x{res[0][1][k]:5.0f}  {k[:60]}"
        if len(res) > 1:
            line += f"   | {res[1][0].get(k, 0.0):8.1f}"
        print(line)
    if len(res) > 1:
        keys = set(res[0][0]) | set(res[1][0])
        diff = sorted(((res[0][0].get(k, 0) - res[1][0].get(k, 0), k) for k in keys))
        print("largest differences (run0 - run1, us/step):")
        for dlt, k in diff[:8] + diff[-8:]:
            print(f"  {dlt:+8.1f}  {k[:70]}")


if __name__ == "__main__":
    main()
