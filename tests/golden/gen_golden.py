"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
(Luka140/paig_reproduction, read-only at /root/reference) on CPU.

Run here (the survey container) only:   python tests/golden/gen_golden.py
The GPU box never sees /root/reference; it gets only the .npz files this
script writes.  Nothing from the reference is copied: the script imports it,
feeds it synthetic inputs + deterministic weights and records outputs.

Harness adaptations, none of which edit the reference:
  * ``tensorflow`` is imported but unused (nn/network/stn.py:1) -> empty stub.
  * ``torchvision.transforms.Resize`` (nn/network/blocks.py:4) -> stub whose
    forward is ``F.interpolate(bilinear, align_corners=False, antialias=True)``,
    the torchvision>=0.17 tensor path.
  * extra_valid/test fns (visualisation, needs moviepy) are cleared.
  * "fresh" loss mode: ``m.output = m(x)`` before ``compute_loss`` (undoes Q1).
  * gravity: ``cell.A`` is recomputed from g, m before the forward (Q4).
"""
import importlib.machinery
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from weights import golden_state  # noqa: E402
from paig_reproduction_amd.nn.datasets.synth import render_sequences, as_model_input  # noqa: E402


def _install_shims():
    tf = types.ModuleType("tensorflow")
    tf.__spec__ = importlib.machinery.ModuleSpec("tensorflow", None)
    sys.modules["tensorflow"] = tf

    class InterpolationMode:
        BILINEAR = "bilinear"

    class Resize(torch.nn.Module):
        def __init__(self, size, interpolation=None):
            super().__init__()
            self.size = tuple(size)

        def forward(self, x):
            return F.interpolate(x, size=self.size, mode="bilinear", align_corners=False, antialias=True)

    tv = types.ModuleType("torchvision")
    tv.__spec__ = importlib.machinery.ModuleSpec("torchvision", None)
    tvt = types.ModuleType("torchvision.transforms")
    tvt.__spec__ = importlib.machinery.ModuleSpec("torchvision.transforms", None)
    tvt.Resize = Resize
    tvt.InterpolationMode = InterpolationMode
    tv.transforms = tvt
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tvt


# name -> (task, cell, seq_len, input_steps, pred_steps, size, B, ae, alt_vel)
# presets: runners/torch_run_physics.py:49-75
CONFIGS = {
    "spring_s12": ("spring_color", "spring_ode_cell", 12, 4, 6, 32, 3, 3.0, False),
    "spring_s50": ("spring_color", "spring_ode_cell", 50, 4, 6, 32, 2, 3.0, False),
    "spring_altvel": ("spring_color", "spring_ode_cell", 12, 4, 6, 32, 2, 3.0, True),
    "bouncing_s12": ("bouncing_balls", "bouncing_ode_cell", 12, 4, 6, 32, 2, 2.0, False),
    "3bp_s20": ("3bp_color", "gravity_ode_cell", 20, 4, 12, 36, 2, 5.0, False),
    "mnist_s12": ("mnist_spring_color", "spring_ode_cell", 12, 3, 7, 64, 2, 3.0, False),
}

BIG = 20000  # grads with more elements are stored as summaries


def run_config(name, seed=0):
    from nn.network.physics_models import PhysicsNet

    task, cell, seq_len, ins, pred, size, B, ae, alt_vel = CONFIGS[name]
    torch.manual_seed(0)
    m = PhysicsNet(task, 100, 1, cell, seq_len, ins, pred, ae, alt_vel, True, size * size,
                   "conv_encoder", "conv_st_decoder", device=torch.device("cpu"))
    m.extra_valid_fns.clear()
    m.extra_test_fns.clear()
    sd = m.state_dict()
    shapes = {k: (tuple(v.shape), str(v.numpy().dtype)) for k, v in sd.items()}
    gs = golden_state(shapes, seed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in gs.items()})
    if cell == "gravity_ode_cell":
        m.rollout_cell.A = torch.exp(m.rollout_cell.g) * torch.exp(2 * m.rollout_cell.m)

    u8 = render_sequences(task, B, seq_len, seed=100 + seed)
    x = torch.from_numpy(as_model_input(u8)).requires_grad_(True)
    m.output = m(x)
    train_loss, (pred_l, extrap_l, recons_l) = m.compute_loss()
    # true prediction loss (before the in-place Q2 aliasing) recomputed from outputs
    tgt = x.detach()[:, ins:]
    L = ((tgt - m.output.detach()) ** 2).sum(dim=[2, 3, 4])
    pred_true = L[:, :pred].mean()
    m.zero_grad(set_to_none=True)
    train_loss.backward()

    out = {
        "input_u8": u8,
        "enc_pos": m.enc_pos.detach().numpy(),
        "enc_masks": m.enc_masks.detach().numpy(),
        "recons_out": m.recons_out.detach().numpy(),
        "output_seq": m.output.detach().numpy(),
        "pos_vel_seq": m.pos_vel_seq.detach().numpy(),
        "loss_train": np.float64(train_loss.item()),
        "loss_pred_aliased": np.float64(pred_l.item()),
        "loss_pred_true": np.float64(pred_true.item()),
        "loss_extrap": np.float64(extrap_l.item()),
        "loss_recons": np.float64(recons_l.item()),
    }
    grad_keys = []
    for k, p in m.named_parameters():
        if p.grad is None:
            continue
        grad_keys.append(k)
        g = p.grad.detach().numpy()
        if g.size <= BIG:
            out["grad/" + k] = g
        else:
            g2 = g.reshape(g.shape[0], -1)
            out["gradsum0/" + k] = g2.sum(axis=0)
            out["gradsum1/" + k] = g2.sum(axis=1)
            out["gradslice/" + k] = g2[:64, :64]
            out["gradnorm/" + k] = np.float64(np.linalg.norm(g2.astype(np.float64)))
    out["grad_keys"] = np.array(grad_keys)
    out["state_keys"] = np.array(list(sd.keys()))
    out["state_shapes"] = np.array(["%s|%s|%s" % (k, ",".join(str(d) for d in v[0]), v[1]) for k, v in shapes.items()])
    out["config"] = np.array([task, cell, str(seq_len), str(ins), str(pred), str(size), str(B), str(ae),
                              str(int(alt_vel))])
    return out


def main():
    _install_shims()
    sys.path.insert(0, REF)
    torch.set_num_threads(4)
    names = sys.argv[1:] or list(CONFIGS)
    for name in names:
        o = run_config(name)
        path = os.path.join(HERE, f"golden_{name}.npz")
        np.savez_compressed(path, **o)
        print(f"{name}: wrote {path} ({os.path.getsize(path) / 1e3:.0f} kB) "
              f"train={o['loss_train']:.4f} recons={o['loss_recons']:.4f} "
              f"extrap={o['loss_extrap']:.4f} grads={len(o['grad_keys'])}")


if __name__ == "__main__":
    main()
