"""Per-kernel average durations of two rocprofv3 kernel_stats.csv files.
usage: python tools/prof_diff.py A.csv B.csv [rows]"""
import csv
import sys


def load(p):
    d = {}
    for r in csv.DictReader(open(p)):
        d[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3)
    return d


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    keys = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (1, 0))[1], b.get(k, (1, 0))[1]))
    ta, tb = sum(v[1] for v in a.values()), sum(v[1] for v in b.values())
    print(f"total {ta:12.0f} us -> {tb:12.0f} us")
    for k in keys[:n]:
        ca, ua = a.get(k, (0, 0.0))
        cb, ub = b.get(k, (0, 0.0))
        print(f"{ua / max(ca, 1):10.1f} {ub / max(cb, 1):10.1f} us/launch  {ua:10.0f} {ub:10.0f} us  {k[:70]}")


if __name__ == "__main__":
    main()
