"""Time the REFERENCE's own training step against the oracle restatement on
this (build) container's CPU, so bench.py's cpu_baseline -- which times the
oracle (the reference is not on the GPU box) -- can be related to the
reference's code path.

Run here only (needs /root/reference; nothing of it is copied):
    python tools/time_reference.py [threads=8] [seconds=20]

Both run fresh-mode train steps, alternated step by step (median of each), (forward, compute_loss, backward: the
reference's nn/network/base.py:139-151 minus the optimizer) of spring_color
B=100 at seq_len 50 (config #1) and 12 (the reference's default), on the
same synthetic batch, with the same torch thread count.  The reference is
imported with tests/golden/gen_golden.py's shims (an empty tensorflow, the
torchvision Resize as F.interpolate) and its extra_*_fns cleared.
Differences: the reference recomputes the decoder sources (the three
VariableFromNetwork MLPs) in every one of its R+1 conv_st_decoder calls
(nn/network/physics_models.py:163,168,185); the oracle forms them once per
step (Q12), as the HIP path does.  Writes profiles/cpu_reference_vs_oracle.json.
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests", "golden")]


def _alternating(fa, fb, budget):
    """Steps of a and b alternated (a, b, a, b, ...) until 2 x budget seconds
    have passed: load drift on a shared host hits both alike.  Returns the
    median step time of each."""
    fa()   # warm-up
    fb()
    ta, tb = [], []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2 * budget or len(ta) < 3:
        for f, acc in ((fa, ta), (fb, tb)):
            t = time.perf_counter()
            f()
            acc.append(time.perf_counter() - t)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    return med(ta), med(tb), len(ta)


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    budget = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    torch.set_num_threads(threads)
    import gen_golden
    from oracle import physics_oracle as O
    from paig_reproduction_amd.nn.datasets.synth import as_model_input, render_sequences
    gen_golden._install_shims()
    sys.path.insert(0, "/root/reference")
    from nn.network.physics_models import PhysicsNet as RefNet

    B = 100
    res = {"threads": threads, "batch": B, "task": "spring_color", "rows": {}}
    for sl in (50, 12):
        u8 = render_sequences("spring_color", B, sl, seed=1)
        x = torch.from_numpy(as_model_input(u8))
        torch.manual_seed(0)
        ref = RefNet("spring_color", 100, 1, "spring_ode_cell", sl, 4, 6, 3.0, False, True, 32 * 32,
                     "conv_encoder", "conv_st_decoder", device=torch.device("cpu"))
        ref.extra_valid_fns.clear()
        ref.extra_test_fns.clear()
        state = {k: v.detach().clone() for k, v in ref.state_dict().items()}

        def ref_step():
            ref.output = ref(x)
            loss, _ = ref.compute_loss()
            ref.zero_grad(set_to_none=True)
            loss.backward()

        cfg = O.Cfg("spring_color", "spring_ode_cell", sl, 4, 6, 32, 3.0)

        def oracle_step():
            O.train_step(state, cfg, x)

        tr, to, n = _alternating(ref_step, oracle_step, budget)
        row = {"reference_seqs_per_s": round(B / tr, 2), "oracle_seqs_per_s": round(B / to, 2),
               "steps_each": n, "reference_median_s": round(tr, 3), "oracle_median_s": round(to, 3)}
        row["oracle_over_reference"] = round(row["oracle_seqs_per_s"] / row["reference_seqs_per_s"], 3)
        res["rows"][f"seq{sl}"] = row
        print(f"seq_len {sl}: {row}", flush=True)
    try:
        res["cpu"] = next(line.split(":", 1)[1].strip() for line in open("/proc/cpuinfo")
                          if line.startswith("model name"))
    except (OSError, StopIteration):
        res["cpu"] = "unknown"
    out = os.path.join(REPO, "profiles", "cpu_reference_vs_oracle.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
