"""Summarise a bench.py --profile-ops table (per-op HIP-event timings)."""
import collections
import re
import sys

NAMES = {1: 'conv_fwd', 2: 'dgrad', 3: 'wgrad', 4: 'convT', 5: 'pool', 6: 'poolbwd', 7: 'tail',
         8: 'tailbwd', 9: 'bnupd', 10: 'final', 12: 'memset'}
rows = []
for line in open(sys.argv[1]):
    m = re.match(r'(\w+)\s+(\d+)\s+([\d.]+)us\s+([\d.]+)%\s+(\S*)\s*kind=(\d+) flops=(\d+) bytes=(\d+)', line)
    if m:
        rows.append((m.group(1), int(m.group(2)), float(m.group(3)), m.group(5), int(m.group(6))))
tot = sum(r[2] for r in rows)
print('total us', round(tot), 'ops', len(rows))
k = collections.defaultdict(float)
n = collections.Counter()
for r in rows:
    k[r[4]] += r[2]
    n[r[4]] += 1
for kk, v in sorted(k.items(), key=lambda x: -x[1]):
    print(f'{NAMES.get(kk, kk):9s} {v:8.0f}us  n={n[kk]:3d}  avg={v / n[kk]:6.1f}')
for lo, hi in ((0, 10), (10, 20), (20, 40), (40, 80), (80, 1e9)):
    s = [r for r in rows if lo <= r[2] < hi]
    print(f'ops {lo}-{hi}us: {len(s):3d} sum {sum(r[2] for r in s):7.0f}')
