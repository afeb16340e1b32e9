"""Per-step summary of a `rocprofv3 --kernel-trace --stats` kernel_stats.csv.

usage: python tools/prof_summary.py <kernel_stats.csv> [steps_profiled] [top_n]
"""
import csv
import re
import sys


def main():
    # at::cuda::spin_kernel is the probe's queue filler (bench.py KernelProbe:
    # keeps the GPU ahead of the host so HIP events time the kernels), not work
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "spin_kernel" not in r["Name"]]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
        name = re.sub(r"\(.*", "", name)
        t = float(r["TotalDurationNs"])
        print("%6.2f%% %7.1fus/step n=%5s avg=%7.1fus %s" % (
            100 * t / tot, t / 1e3 / steps, r["Calls"], float(r["AverageNs"]) / 1e3, name[:90]))
    print("%.3f ms/step GPU busy" % (tot / 1e6 / steps))


if __name__ == "__main__":
    main()
