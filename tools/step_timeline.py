"""One training step of a rocprofv3 kernel trace as a timeline: start offset, duration,
queue and name of every kernel between two Adam launches (the step-th from the end).

    python tools/step_timeline.py gpurun_out/prof_TAG [step_from_end=2] [--tail N]
"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 2
    tail = int(sys.argv[sys.argv.index("--tail") + 1]) if "--tail" in sys.argv else 0
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         n.split("(")[0].strip(), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if "adam" in r[3] or "step_tail" in r[3]]
    a, b = adam[-k - 1] + 1, adam[-k] + 1
    step = rows[a:b]
    t0 = step[0][0]
    print(f"step span {(step[-1][1] - t0) / 1e3:.1f} us, {len(step)} kernels")
    for s, e, q, n, g in step[-tail:] if tail else step:
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q}  {n[:60]:60s} wg {g}")


if __name__ == "__main__":
    main()
