"""HBM traffic per kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D -o f -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d D -o w -- python3 bench.py ...
    python tools/pmc_traffic.py f_counter_collection.csv w_counter_collection.csv out.json \
        [--steps S --task T --batch B --seq_len L --probe TAG=KERNEL ... --command CMD]

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled; WRITE_SIZE is taken as is.  Infinity-Cache hits are counted too, so
this is memory-side (L2 miss) traffic, an upper bound on HBM bytes.
"""
import argparse
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.sub(r"\(.*", "", name).strip()


def load(path, counter):
    per = defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        # launches of one kernel with different grids (e.g. the decoder over
        # rollout and reconstruction frames) are kept apart: "name @grid"
        k = short(r["Kernel_Name"]) + " @" + r["Grid_Size"]
        per[k].append(float(r["Counter_Value"]) * 1024.0)
        meta[k] = {"vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                   "lds": int(r["LDS_Block_Size"]), "wg": int(r["Workgroup_Size"])}
    return per, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, default=1, help="training steps the profiled run executed")
    ap.add_argument("--task", default="spring_color")
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--seq_len", type=int, default=50)
    ap.add_argument("--conv_math", default="split")
    ap.add_argument("--probe", action="append", default=[],
                    help="TAG=KERNEL @GRID: bench.py probe tag -> kernel name and grid (a key of 'kernels')")
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    f, meta = load(a.fetch, "FETCH_SIZE")
    w, _ = load(a.write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fr = 2.0 * sum(f.get(k, [0])) / max(len(f.get(k, [])), 1)
        wr = sum(w.get(k, [0])) / max(len(w.get(k, [])), 1)
        res[k] = {"launches": len(f.get(k, [])), "fetch_bytes_raw": fr / 2, "fetch_bytes": fr, "write_bytes": wr,
                  "traffic_bytes": fr + wr, **meta.get(k, {})}
    probes = dict(p.split("=", 1) for p in a.probe)
    json.dump({"correction": "fetch x2 (gfx950 FETCH_SIZE halving), KiB -> bytes", "command": a.command,
               "config": {"task": a.task, "batch": a.batch, "seq_len": a.seq_len, "conv_math": a.conv_math}, "steps_profiled": a.steps,
               "probe_kernels": probes, "kernels": res}, open(a.out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes"] * kv[1]["launches"])[:25]:
        print("%-70s n=%4d  fetch %9.2f MB  write %9.2f MB" % (k[:70], v["launches"], v["fetch_bytes"] / 1e6,
                                                                 v["write_bytes"] / 1e6))


if __name__ == "__main__":
    main()
