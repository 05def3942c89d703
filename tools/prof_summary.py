"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) or kernel_stats.csv into a
plain-text table: kernel, calls, total us, average us, share.

    python tools/prof_summary.py gpurun_out/prof_X/run_results.db > profiles/X_kernel_stats.txt
"""
import csv
import sqlite3
import sys


def rows_from(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4]))  # view is in us
                for r in c.execute("select name,total_calls,total_duration,average,percentage "
                                   "from top_kernels")]
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main():
    rows = rows_from(sys.argv[1])
    print(f"# rocprofv3 --kernel-trace --stats summary of {sys.argv[1].split('gpurun_out/')[-1]}")
    print(f"{'calls':>7} {'total_us':>12} {'avg_us':>10} {'pct':>6}  kernel")
    for name, calls, tot, avg, pct in rows:
        short = name.replace("(anonymous namespace)::", "")
        print(f"{calls:7d} {tot:12.1f} {avg:10.3f} {pct:6.2f}  {short[:150]}")


if __name__ == "__main__":
    main()
