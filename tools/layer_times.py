"""Per-launch times of every probed kernel of the training step (HIP events
on the launching stream, engine.KernelProbe), for A/B of the conv backward
forms: PAIG_FUSED_BWD=1 (fused layer backward) vs 0 (separate dgrad / wgrad).

    python tools/layer_times.py [--task spring_color --batch 100 --seq_len 50 --steps 5]
Prints one JSON line {tag: avg_us} per mode.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, REPO)
    import numpy as np
    import torch
    from paig_reproduction_amd import engine as E
    from paig_reproduction_amd.nn.datasets.synth import as_model_input, render_sequences
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet
    import bench
    cell, ins, pred, size = bench.TASKS[a.task]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = PhysicsNet(a.task, 100, 1, cell, a.seq_len, ins, pred, 3.0, False, True, size * size, "conv_encoder",
                   "conv_st_decoder", device=dev).to(dev)
    m.conv_math = a.conv_math
    m.build_optimizer(6e-4, "rmsprop", True)
    u8 = render_sequences(a.task, min(a.batch, 64), a.seq_len, seed=1)
    u8 = np.concatenate([u8] * (-(-a.batch // u8.shape[0])), 0)[:a.batch]
    x = torch.from_numpy(as_model_input(u8)).to(dev)
    eng = m._native()

    def step():
        m.output = m(x)
        loss, _ = m.compute_loss()
        m.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        m.optimizer.step()

    for _ in range(3):
        step()
    probe = E.KernelProbe(None)
    eng.probe = probe
    for _ in range(a.steps):
        step()
    eng.probe = None
    s = probe.summaries()
    out = {t: round(v["avg_ms"] * 1e3, 2) for t, v in sorted(s.items())}
    print("LAYER_TIMES " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="spring_color")
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--seq_len", type=int, default=50)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--conv_math", default="split")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    res = {}
    for mode in ("0", "1"):
        env = dict(os.environ, PAIG_FUSED_BWD=mode)
        out = subprocess.run([sys.executable, __file__, "--child"] + sys.argv[1:], env=env, capture_output=True,
                             text=True, timeout=600)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("LAYER_TIMES ")]
        if not line:
            print(out.stdout[-2000:], out.stderr[-3000:])
            raise SystemExit(1)
        res[mode] = json.loads(line[0][len("LAYER_TIMES "):])
    names = sorted(set(res["0"]) | set(res["1"]))
    layers = sorted({t.split(":")[1] for t in names if t.startswith("conv_")}, key=lambda s: int(s[1:]))
    print(f"{'layer':6s} {'dgrad':>8s} {'wgrad':>8s} {'sum':>8s} {'fused':>8s}")
    tot0 = tot1 = 0.0
    for l in layers:
        d = res["0"].get("conv_dgrad:" + l, 0.0)
        w = res["0"].get("conv_wgrad:" + l, 0.0)
        f = res["1"].get("conv_bwd:" + l)
        fd = res["1"].get("conv_dgrad:" + l, 0.0) + res["1"].get("conv_wgrad:" + l, 0.0)
        tot0 += d + w
        tot1 += f if f is not None else fd
        print(f"{l:6s} {d:8.2f} {w:8.2f} {d + w:8.2f} {f if f is not None else fd:8.2f}{'' if f is not None else ' (separate)'}")
    print(f"total conv backward: separate {tot0:.1f} us, fused {tot1:.1f} us")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
