"""Measure the HIP step's distance to the float64 oracle against the fp32
oracle's own distance (tests/envelope.py), for every golden config and conv
arithmetic; writes a JSON table.  Run on the GPU box from the repo root:
    python tools/grad_envelope.py gpurun_out/grad_envelope.json split fp32"""
import json
import os
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
import torch  # noqa: E402
from helpers import GOLDEN  # noqa: E402
from envelope import envelope  # noqa: E402


def main():
    path = sys.argv[1]
    modes = sys.argv[2:] or ["split", "fp32"]
    dev = torch.device("cuda:0")
    table = {}
    for name in GOLDEN:
        for cm in modes:
            rows = envelope(name, cm, dev)
            table[f"{name}/{cm}"] = {k: {"hip_vs_f64": a, "fp32_vs_f64": b, "bar": c} for k, (a, b, c) in rows.items()}
            over = {k: (a, c) for k, (a, b, c) in rows.items() if a > c}
            worst = sorted(rows.items(), key=lambda kv: -kv[1][0] / max(kv[1][2], 1e-30))[:4]
            print(f"{name:14s} {cm:6s} over={len(over):2d} worst(ratio hip/bar): " +
                  " ".join(f"{k}={a:.1e}/{b:.1e}" for k, (a, b, c) in worst), flush=True)
    with open(path, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
