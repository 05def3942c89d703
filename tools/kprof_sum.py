"""Per-kernel GPU durations from a rocprofv3 SQLite trace (rocpd tables)."""
import sqlite3
import sys

for f in sys.argv[1:]:
    c = sqlite3.connect(f)
    q = ("select s.kernel_name, count(*), avg(d.end - d.start), min(d.end - d.start) "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
         "group by s.kernel_name order by 3 desc")
    for name, n, avg, mn in c.execute(q):
        print(f"  {n:5d} avg {avg / 1e3:8.2f} us  min {mn / 1e3:8.2f} us  {name[:90]}")
