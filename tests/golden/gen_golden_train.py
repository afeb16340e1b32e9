"""Golden fixtures of the reference's TRAINING loop and eval path, produced by
running the REFERENCE (read-only at /root/reference) on CPU:

  train_traj_<cfg>.npz     10 fresh-mode RMSprop steps (nn/network/base.py:138-152
                     with m.output = m(x)): per-step losses and the
                     final parameters (full when small, else summaries)
  train_refmode_<cfg>.npz  the reference's ACTUAL step (quirk Q1, base.py:141-143 vs
                     :195): an eval forward sets self.output under no_grad,
                     then train steps whose loss reads that stale output
  train_eval_<cfg>.npz     the test phase (runners/torch_run_physics.py:101-117): a
                     model built at test_seq_len, eval_performance over a
                     small test set (Q15: < 100 examples -> one whole-set batch)

Run here only:   python tests/golden/gen_golden_train.py
The GPU box gets only the .npz files.  Same shims / adaptations as
gen_golden.py; weights from weights.py (regenerated, not stored).
"""
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (shims, CONFIGS, paths)
from weights import golden_state  # noqa: E402
from paig_reproduction_amd.nn.datasets.synth import render_sequences, as_model_input  # noqa: E402

BIG = 20000
LR = 1e-3          # runners/torch_run_physics.py:15 --base_lr default
TRAJ_STEPS = 10


def _model(name, seq_len=None):
    from nn.network.physics_models import PhysicsNet
    task, cell, sl, ins, pred, size, B, ae, alt = G.CONFIGS[name]
    sl = seq_len or sl
    torch.manual_seed(0)
    m = PhysicsNet(task, 100, 1, cell, sl, ins, pred, ae, alt, True, size * size, "conv_encoder", "conv_st_decoder",
                   device=torch.device("cpu"))
    m.extra_valid_fns.clear()
    m.extra_test_fns.clear()
    sd = m.state_dict()
    shapes = {k: (tuple(v.shape), str(v.numpy().dtype)) for k, v in sd.items()}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_state(shapes, 0).items()})
    return m, shapes, (task, cell, sl, ins, pred, size, B, ae, alt)


def _fix_gravity(m):
    if hasattr(m.rollout_cell, "g"):   # Q4: recompute A from g, m before every forward
        m.rollout_cell.A = torch.exp(m.rollout_cell.g) * torch.exp(2 * m.rollout_cell.m)


def _params(out, m, prefix):
    for k, p in m.named_parameters():
        v = p.detach().numpy()
        if v.size <= BIG:
            out[f"{prefix}/{k}"] = v.copy()
        else:
            v2 = v.reshape(v.shape[0], -1).astype(np.float64)
            out[f"{prefix}sum0/{k}"] = v2.sum(0)
            out[f"{prefix}sum1/{k}"] = v2.sum(1)
            out[f"{prefix}slice/{k}"] = v.reshape(v.shape[0], -1)[:64, :64].copy()
            out[f"{prefix}norm/{k}"] = np.float64(np.linalg.norm(v2))


def _grads(out, m):
    keys = []
    for k, p in m.named_parameters():
        if p.grad is None:
            continue
        keys.append(k)
        g = p.grad.detach().numpy()
        if g.size <= BIG:
            out["grad/" + k] = g.copy()
        else:
            g2 = g.reshape(g.shape[0], -1)
            out["gradsum0/" + k] = g2.sum(axis=0)
            out["gradsum1/" + k] = g2.sum(axis=1)
            out["gradslice/" + k] = g2[:64, :64].copy()
            out["gradnorm/" + k] = np.float64(np.linalg.norm(g2.astype(np.float64)))
    out["grad_keys"] = np.array(keys)


def _meta(out, shapes, cfg):
    task, cell, sl, ins, pred, size, B, ae, alt = cfg
    out["state_shapes"] = np.array(["%s|%s|%s" % (k, ",".join(str(d) for d in v[0]), v[1]) for k, v in shapes.items()])
    out["config"] = np.array([task, cell, str(sl), str(ins), str(pred), str(size), str(B), str(ae), str(int(alt))])


def _losses(m):
    tl, (p, e, r) = m.compute_loss()
    return tl, [float(tl), float(p), float(e), float(r)]


def traj(name):
    """TRAJ_STEPS fresh-mode RMSprop steps over two alternating batches."""
    m, shapes, cfg = _model(name)
    task, cell, sl, ins, pred, size, B, ae, alt = cfg
    u8 = [render_sequences(task, B, sl, seed=200 + i) for i in range(2)]
    m.build_optimizer(LR, "rmsprop", True)
    losses = []
    for s in range(TRAJ_STEPS):
        _fix_gravity(m)
        x = torch.from_numpy(as_model_input(u8[s % 2])).requires_grad_(True)
        m.output = m(x)
        tl, lv = _losses(m)
        losses.append(lv)
        m.optimizer.zero_grad(set_to_none=True)
        tl.backward()
        m.optimizer.step()
    out = {"input_u8_0": u8[0], "input_u8_1": u8[1], "losses": np.array(losses), "lr": np.float64(LR),
           "steps": np.int64(TRAJ_STEPS)}
    _params(out, m, "final")
    _meta(out, shapes, cfg)
    return out


def refmode(name):
    """Quirk Q1: eval forward (no_grad) sets self.output; the train steps'
    losses read it while their gradients flow only through the current
    forward's reconstruction term."""
    m, shapes, cfg = _model(name)
    task, cell, sl, ins, pred, size, B, ae, alt = cfg
    u8_eval = render_sequences(task, B, sl, seed=210)
    u8 = [render_sequences(task, B, sl, seed=211 + i) for i in range(2)]
    m.build_optimizer(LR, "rmsprop", True)
    with torch.no_grad():
        _fix_gravity(m)
        m.output = m.conv_feedforward(torch.from_numpy(as_model_input(u8_eval)))
    losses, out = [], {}
    for s in range(2):
        _fix_gravity(m)
        x = torch.from_numpy(as_model_input(u8[s])).requires_grad_(True)
        m.forward(x)                      # result discarded (base.py:142)
        tl, lv = _losses(m)               # reads the stale self.output (Q1)
        losses.append(lv)
        m.optimizer.zero_grad(set_to_none=True)
        tl.backward()
        if s == 0:
            _grads(out, m)
        m.optimizer.step()
    out.update({"input_u8_eval": u8_eval, "input_u8_0": u8[0], "input_u8_1": u8[1], "losses": np.array(losses),
                "lr": np.float64(LR)})
    _params(out, m, "final")
    _meta(out, shapes, cfg)
    return out


def evalpass(name, test_seq_len, n_test):
    """The test phase: the model rebuilt at test_seq_len, eval_performance over
    a test set of n_test (< 100: one whole-set batch, Q15) sequences."""
    from nn.datasets.iterators import DataIterator
    m, shapes, cfg = _model(name, test_seq_len)
    task, cell, sl, ins, pred, size, B, ae, alt = cfg
    u8 = render_sequences(task, n_test, sl, seed=220)
    x = as_model_input(u8)
    m.test_iterator = DataIterator(x)
    np.random.seed(0)
    _fix_gravity(m)
    with tempfile.TemporaryDirectory() as d:
        m.save_dir = d
        metrics = m.eval_performance(100, type="test")
    with torch.no_grad():
        _fix_gravity(m)
        out_seq = m.conv_feedforward(torch.from_numpy(x))
        tl, lv = _losses(m)
    out = {"input_u8": u8, "output_seq": out_seq.numpy(), "pos_vel_seq": m.pos_vel_seq.numpy(),
           "losses": np.array(lv)}
    for k, v in metrics.items():
        out["metric/" + k] = np.asarray(v, dtype=np.float64)
    _meta(out, shapes, cfg)
    return out


JOBS = {
    "traj_spring_s12": lambda: traj("spring_s12"),
    "traj_mnist_s12": lambda: traj("mnist_s12"),
    "refmode_spring_s12": lambda: refmode("spring_s12"),
    "eval_spring_s30": lambda: evalpass("spring_s12", 30, 5),
    "eval_3bp_s40": lambda: evalpass("3bp_s20", 40, 3),
}


def main():
    G._install_shims()
    sys.path.insert(0, G.REF)
    torch.set_num_threads(4)
    for name in sys.argv[1:] or list(JOBS):
        o = JOBS[name]()
        path = os.path.join(HERE, f"train_{name}.npz")
        np.savez_compressed(path, **o)
        print(f"{name}: wrote {path} ({os.path.getsize(path) / 1e3:.0f} kB) losses[0]={np.asarray(o['losses'])[0]}")


if __name__ == "__main__":
    main()
