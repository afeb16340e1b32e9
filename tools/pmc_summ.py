"""Per-kernel averages of every counter in rocprofv3 --pmc CSV files.

usage: python tools/pmc_summ.py DIR_OR_CSV... [--filter substr] [--json out.json]
Launches of one kernel with different grids are kept apart ("name @grid").
FETCH_SIZE is doubled (gfx950 reports half of wide coalesced reads,
MI355X_MICROARCH.md HBM section); FETCH_SIZE / WRITE_SIZE are KiB -> bytes.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*", "", name).strip()


def main():
    args = [a for a in sys.argv[1:]]
    filt, out = "", None
    if "--filter" in args:
        i = args.index("--filter")
        filt = args[i + 1]
        del args[i:i + 2]
    if "--json" in args:
        i = args.index("--json")
        out = args[i + 1]
        del args[i:i + 2]
    files = []
    for a in args:
        files += sorted(glob.glob(os.path.join(a, "**", "*counter_collection.csv"), recursive=True)) if os.path.isdir(a) else [a]
    vals = defaultdict(lambda: defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"]) + " @" + r["Grid_Size"]
            if filt and filt not in k:
                continue
            v = float(r["Counter_Value"])
            c = r["Counter_Name"]
            if c == "FETCH_SIZE":
                v *= 2 * 1024
            elif c == "WRITE_SIZE":
                v *= 1024
            vals[k][c].append(v)
    res = {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"launches": max(len(v) for v in cs.values())}
           for k, cs in vals.items()}
    for k, cs in sorted(res.items()):
        print(k)
        wc = cs.get("SQ_WAVE_CYCLES")
        for c, v in sorted(cs.items()):
            frac = f"  ({v / wc:.3f} of wave cycles)" if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
            print(f"    {c:28s} {v:16.1f}{frac}")
    if out:
        json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
