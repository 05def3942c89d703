"""Compare two per-op tables (bench.py --profile-ops): python tools/opcmp.py A B [n]."""
import sys


def load(p):
    d = {}
    for l in open(p):
        f = l.split()
        d[(f[0], f[1], f[4] if len(f) > 4 else '')] = float(f[2].replace('us', ''))
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 15
print(f"total {sum(a.values()):.1f} -> {sum(b.values()):.1f} us over {len(a)} / {len(b)} ops")
rows = sorted((b[k] - a[k], a[k], b[k], k) for k in a if k in b)
for r in rows[:n] + [None] + rows[-n:]:
    print('...' if r is None else f"{r[0]:+7.1f}  {r[1]:7.1f} -> {r[2]:7.1f}  {' '.join(r[3])}")
