"""Critical-path view of one graph-replayed step from a rocprofv3
kernel_trace.csv: kernels of the last complete step in start order with
their queue, start offset, duration and the idle gap before them (time with
no kernel running on any queue), plus the totals.

usage: python tools/timeline.py <kernel_trace.csv> [first_kernel_substring]
The step boundary is the first kernel whose name contains the substring
(default gather_u8_f32_k, the step's first launch)."""
import csv
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", n)[:70]


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "spin_kernel" not in r["Kernel_Name"]]
    key = sys.argv[2] if len(sys.argv) > 2 else "gather_u8_f32_k"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
    a, b = starts[-3], starts[-2]   # a complete step well inside the timed loop
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    t_end = int(rows[b]["Start_Timestamp"])
    busy_end = t0
    idle = 0
    print(f"{'start':>8} {'dur':>7} {'gap':>6} q  kernel")
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(0, s - busy_end)
        idle += gap
        busy_end = max(busy_end, e)
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {gap / 1e3:6.1f} {r['Queue_Id']:>2} {short(r['Kernel_Name'])}")
    idle += max(0, t_end - busy_end)
    print(f"step {(t_end - t0) / 1e3:.1f} us, idle (no kernel on any queue) {idle / 1e3:.1f} us, "
          f"{len(step)} kernels")


if __name__ == "__main__":
    main()
