"""Main-queue gaps of one training step in a rocprofv3 kernel trace: which kernel ends just
before each gap on the main queue, and what runs on the other queues meanwhile (a join
waiting for a side stream shows up as a gap that ends when a side kernel ends).
  python tools/ktrace_gaps.py gpurun_out/prof_X/run_kernel_trace.csv [min_gap_us]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
      re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")))
     for r in rows]
k.sort()
# one step = the last occurrence of the step's first kernel (the loss kernel ends it):
# take the span between the last two head_fwd launches
heads = [i for i, x in enumerate(k) if x[3].startswith("head_fwd")]
assert len(heads) >= 3, "no training steps in the trace"
a, b = heads[-3], heads[-2]
step = k[a:b]
q = defaultdict(list)
for x in step:
    q[x[2]].append(x)
main = max(q, key=lambda z: len(q[z]))
t0 = step[0][0]
print(f"step span {(step[-1][1] - t0) / 1e3:.1f} us, kernels {len(step)}")
for z, v in sorted(q.items()):
    busy = sum(e - s for s, e, _, _ in v)
    print(f"  queue {z}{' (main)' if z == main else ''}: {len(v)} kernels, busy {busy / 1e3:.1f} us")
m = q[main]
tot = 0.0
for (s0, e0, _, n0), (s1, e1, _, n1) in zip(m, m[1:]):
    gap = (s1 - e0) / 1e3
    if gap < mn:
        continue
    tot += gap
    ends = [x[3] for x in step if x[2] != main and e0 <= x[1] <= s1 + 500]
    print(f"{(e0 - t0) / 1e3:8.1f} gap {gap:6.1f} us after {n0[:40]:40s} before {n1[:40]:40s} side ends: {ends[:3]}")
print(f"gaps >= {mn} us on the main queue: {tot:.1f} us")

# instants when no kernel runs on any queue (launch/dependency latency on the step's path)
ev = sorted((s, e, n) for s, e, _, n in step)
idle, cur_end, last = [], ev[0][1], ev[0][2]
for s, e, n in ev[1:]:
    if s > cur_end:
        idle.append(((s - cur_end) / 1e3, (cur_end - t0) / 1e3, last, n))
    if e > cur_end:
        cur_end, last = e, n
print(f"all-queue idle: {sum(g for g, *_ in idle):.1f} us in {len(idle)} gaps")
for g, at, a_, b_ in sorted(idle, reverse=True)[:25]:
    print(f"  {at:8.1f} idle {g:5.1f} us after {a_[:40]:40s} before {b_[:40]}")
