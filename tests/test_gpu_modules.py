"""The reference's submodules called one at a time, as its callers do
(SURVEY §8 B1): forward values and gradients of the HIP standalone forwards
(nn/network/native_modules.py) against the oracle (tests/golden weights and
inputs; the oracle is pinned to the reference by test_oracle_golden.py):

  VariableFromNetwork()               blocks.py:318-322
  ConvolutionalEncoder(frames)        blocks.py:77-103
  ShallowUNet(frames) / UNet(frames)  blocks.py:278-308 / :172-237
  VelocityEncoder(positions)          blocks.py:31-49
  <cell>(pos, vel)                    cells.py:31-106
  conv_st_decoder(pos) + transf_contents / transf_masks   physics_models.py:151-199
  stn(U, theta, size)                 stn.py:5-16 (vs aten affine_grid + grid_sample fp32)

Gradients: of sum(out * R) for a fixed random R, w.r.t. the module's
parameters and its differentiable inputs.  Bar: 1e-4 normwise (north star).
The U-Net gradients of the encoder / U-Net calls are bounded by the fp32
envelope instead (tests/envelope.py): near-tie max-pool / ReLU decisions of
these inputs flip under one-ulp weight changes, so even honest fp32 runs
differ by more than 1e-4 there; the bar is ENVELOPE_K times the furthest
ensemble member (at least 1e-4).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import load_golden, golden_weights, rel_err
from envelope import ENVELOPE_K, _ulp_perturbed
from oracle import physics_oracle as O

pytestmark = pytest.mark.gpu
RT = 1e-4
DEV = torch.device("cuda:0")


def _setup(name):
    from test_gpu_parity import _model
    z = load_golden(name)
    cfg, _ = O.cfg_from_golden(z)
    state = golden_weights(z)
    m = _model(z, DEV)
    x = O.input_from_u8(z["input_u8"])
    return z, cfg, state, m, x


def _leaf(state, keys):
    return {k: (v.detach().clone().requires_grad_(True) if k in keys else v) for k, v in state.items()}


def _R(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g)


def _check_grads(m, P, keys, what, bars=None):
    pd = dict(m.named_parameters())
    for k in keys:
        assert pd[k].grad is not None, f"{what}: no grad for {k}"
        e = rel_err(pd[k].grad, P[k].grad)
        bar = RT if bars is None else bars[k]
        assert e <= bar, f"{what}: grad {k} {e:.2e} > {bar:.2e}"


def _envelope_bars(state, keys, grads_of, P, members=10):
    """Per-parameter bars: ENVELOPE_K x the furthest of ``members`` oracle
    runs on one-ulp-perturbed weights from the unperturbed oracle's grads."""
    worst = {k: 0.0 for k in keys}
    torch.set_num_threads(8)
    for seed in range(members):
        Q = _leaf(_ulp_perturbed(state, seed), keys)
        g = grads_of(Q)
        for k in keys:
            worst[k] = max(worst[k], rel_err(g[k], P[k].grad))
    return {k: max(ENVELOPE_K * v, RT) for k, v in worst.items()}


def test_variable_from_network():
    z, cfg, state, m, x = _setup("spring_s12")
    K, h = cfg.n_objs, cfg.tmpl
    out = m.var_net_template()
    assert tuple(out.shape) == (K, 1, h, h)
    keys = [k for k in state if k.startswith("var_net_template.")]
    P = _leaf(state, keys)
    ref = O.vfn(P, "var_net_template", [K, 1, h, h])
    assert rel_err(out, ref) <= RT
    R = _R(out.shape, 1)
    m.zero_grad(set_to_none=True)
    (out * R.to(DEV)).sum().backward()
    (ref * R).sum().backward()
    torch.cuda.synchronize()
    _check_grads(m, P, keys, "vfn")


@pytest.mark.parametrize("name", ["spring_s12", "mnist_s12"])
def test_convolutional_encoder(name):
    z, cfg, state, m, x = _setup(name)
    frames = x[:, :cfg.Te].reshape(-1, 3, cfg.size, cfg.size)
    pos, masks, objs = m.encoder(frames.to(DEV))
    live = "encoder.unet." if cfg.size >= 40 else "encoder.shallow_unet."
    keys = [k for k in state if k.startswith(live) or k.startswith("encoder.l")]
    P = _leaf(state, keys)
    rpos, rmasks, robjs = O.encoder(P, cfg, frames)
    assert rel_err(pos, rpos) <= RT
    assert rel_err(masks, rmasks) <= RT
    assert len(objs) == cfg.n_objs and all(rel_err(a, b) <= RT for a, b in zip(objs, robjs))
    R = _R(pos.shape, 2)
    m.zero_grad(set_to_none=True)
    (pos * R.to(DEV)).sum().backward()
    (rpos * R).sum().backward()
    torch.cuda.synchronize()

    def grads_of(Q):
        (O.encoder(Q, cfg, frames)[0] * R).sum().backward()
        return {k: Q[k].grad for k in keys}
    _check_grads(m, P, keys, "encoder", _envelope_bars(state, keys, grads_of, P))
    # only the encoder's parameters got gradients
    assert all(p.grad is None for k, p in m.named_parameters() if not k.startswith("encoder."))


@pytest.mark.parametrize("name,which", [("spring_s12", "shallow_unet"), ("mnist_s12", "unet")])
def test_unet(name, which):
    z, cfg, state, m, x = _setup(name)
    frames = x[:, :cfg.Te].reshape(-1, 3, cfg.size, cfg.size)
    logits = getattr(m.encoder, which)(frames.to(DEV))
    keys = [k for k in state if k.startswith("encoder." + which + ".")]
    P = _leaf(state, keys)
    ref = (O.shallow_unet if which == "shallow_unet" else O.unet)(P, frames)
    assert rel_err(logits, ref) <= RT
    R = _R(ref.shape, 3)
    m.zero_grad(set_to_none=True)
    (logits * R.to(DEV)).sum().backward()
    (ref * R).sum().backward()
    torch.cuda.synchronize()
    fn = O.shallow_unet if which == "shallow_unet" else O.unet

    def grads_of(Q):
        (fn(Q, frames) * R).sum().backward()
        return {k: Q[k].grad for k in keys}
    _check_grads(m, P, keys, which, _envelope_bars(state, keys, grads_of, P))


@pytest.mark.parametrize("name", ["spring_s12", "spring_altvel"])
def test_velocity_encoder(name):
    z, cfg, state, m, x = _setup(name)
    pos_in = torch.from_numpy(np.asarray(z["enc_pos"])[:, :cfg.input_steps].copy())
    pi = pos_in.to(DEV).requires_grad_(True)
    vel = m.velocity_encoder(pi)
    keys = [k for k in state if k.startswith("velocity_encoder.")]
    P = _leaf(state, keys)
    pr = pos_in.clone().requires_grad_(True)
    ref = O.velocity_encoder(P, cfg, pr)
    assert rel_err(vel, ref) <= RT
    R = _R(ref.shape, 4)
    m.zero_grad(set_to_none=True)
    (vel * R.to(DEV)).sum().backward()
    (ref * R).sum().backward()
    torch.cuda.synchronize()
    _check_grads(m, P, keys, "velocity")
    assert rel_err(pi.grad, pr.grad) <= RT


@pytest.mark.parametrize("name", ["spring_s12", "bouncing_s12", "3bp_s20"])
def test_ode_cell(name):
    z, cfg, state, m, x = _setup(name)
    pv = torch.from_numpy(np.asarray(z["pos_vel_seq"])[:, 0].copy())
    D = cfg.D
    pos, vel = pv[:, :D], pv[:, D:]
    pg, vg = pos.to(DEV).requires_grad_(True), vel.to(DEV).requires_grad_(True)
    p1, v1 = m.rollout_cell(pg, vg)
    keys = {"spring_ode_cell": ["rollout_cell.k", "rollout_cell.equil"], "gravity_ode_cell": ["rollout_cell.g"],
            "bouncing_ode_cell": []}[cfg.cell]
    P = _leaf(state, keys)
    pr, vr = pos.clone().requires_grad_(True), vel.clone().requires_grad_(True)
    rp, rv = O.CELLS[cfg.cell](P, pr, vr)
    assert rel_err(p1, rp) <= RT and rel_err(v1, rv) <= RT
    R1, R2 = _R(rp.shape, 5), _R(rv.shape, 6)
    m.zero_grad(set_to_none=True)
    ((p1 * R1.to(DEV)).sum() + (v1 * R2.to(DEV)).sum()).backward()
    ((rp * R1).sum() + (rv * R2).sum()).backward()
    torch.cuda.synchronize()
    assert rel_err(pg.grad, pr.grad) <= RT and rel_err(vg.grad, vr.grad) <= RT
    _check_grads(m, P, keys, "cell")


def test_conv_st_decoder_and_parts():
    z, cfg, state, m, x = _setup("spring_s12")
    pos = torch.from_numpy(np.asarray(z["enc_pos"]).reshape(-1, cfg.D).copy())
    pg = pos.to(DEV).requires_grad_(True)
    out = m.conv_st_decoder(pg)
    keys = [k for k in state if k.startswith("var_net_")]
    P = _leaf(state, keys)
    pr = pos.clone().requires_grad_(True)
    joint, bg = O.decoder_sources(P, cfg)
    ref = O.st_decoder(cfg, joint, bg, pr)
    assert rel_err(out, ref) <= RT
    # the reference's side-effect attributes (physics_models.py:163-196)
    assert rel_err(m.template, O.vfn(P, "var_net_template", [cfg.n_objs, 1, cfg.tmpl, cfg.tmpl])) <= RT
    rc, rm = O.st_decoder_parts(cfg, joint.detach(), bg.detach(), pos)
    assert len(m.transf_contents) == cfg.n_objs + 1 and len(m.transf_masks) == cfg.n_objs + 1
    for a, b in zip(m.transf_contents, rc):
        assert rel_err(a, b) <= RT
    for a, b in zip(m.transf_masks, rm):
        assert rel_err(a, b) <= RT
    R = _R(ref.shape, 7)
    m.zero_grad(set_to_none=True)
    (out * R.to(DEV)).sum().backward()
    (ref * R).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(pg.grad, pr.grad) <= RT
    _check_grads(m, P, keys, "decoder")


def test_transf_parts_after_forward():
    """After a full forward the attributes describe the last decoder call
    (the last rollout step), as in the reference's loop."""
    z, cfg, state, m, x = _setup("spring_s12")
    m.output = m(x.to(DEV))
    P = _leaf(state, [])
    joint, bg = O.decoder_sources(P, cfg)
    last = torch.from_numpy(np.asarray(z["pos_vel_seq"])[:, -1, :cfg.D].copy())
    rc, rm = O.st_decoder_parts(cfg, joint, bg, last)
    for a, b in zip(m.transf_contents, rc):
        assert rel_err(a, b) <= RT
    for a, b in zip(m.transf_masks, rm):
        assert rel_err(a, b) <= RT


def test_stn_general_affine():
    from paig_reproduction_amd.nn.network.stn import stn
    g = torch.Generator().manual_seed(8)
    U = torch.rand(5, 4, 11, 13, generator=g)
    theta = (torch.eye(2, 3).expand(5, 2, 3) + 0.3 * torch.randn(5, 2, 3, generator=g)).contiguous()
    Ug, tg = U.to(DEV).requires_grad_(True), theta.to(DEV).requires_grad_(True)
    out = stn(Ug, tg, (9, 7))
    Ur, tr = U.clone().requires_grad_(True), theta.clone().requires_grad_(True)
    ref = F.grid_sample(Ur, F.affine_grid(tr, (5, 4, 9, 7), align_corners=False), align_corners=False)
    assert rel_err(out, ref) <= 1e-5
    R = _R(ref.shape, 9)
    (out * R.to(DEV)).sum().backward()
    (ref * R).sum().backward()
    torch.cuda.synchronize()
    assert rel_err(Ug.grad, Ur.grad) <= 1e-5
    assert rel_err(tg.grad, tr.grad) <= 1e-4


def test_stn_float64_theta():
    """A float64 theta (the reference's physics-derived thetas are fp64, Q9):
    the grid is formed in fp64 and cast to fp32 before sampling, as
    F.affine_grid in theta's dtype followed by grid.float() (stn.py:12-14);
    checked against those aten ops on the CPU (no fixture covers stn)."""
    from paig_reproduction_amd.nn.network.stn import stn
    g = torch.Generator().manual_seed(12)
    U = torch.rand(4, 3, 16, 16, generator=g)
    theta = (torch.eye(2, 3, dtype=torch.float64).expand(4, 2, 3)
             + 0.3 * torch.randn(4, 2, 3, generator=g, dtype=torch.float64)).contiguous()
    Ug, tg = U.to(DEV).requires_grad_(True), theta.to(DEV).requires_grad_(True)
    out = stn(Ug, tg, (32, 32))
    Ur, tr = U.clone().requires_grad_(True), theta.clone().requires_grad_(True)
    grid = F.affine_grid(tr, (4, 3, 32, 32), align_corners=False)
    ref = F.grid_sample(Ur, grid.float(), align_corners=False)
    assert rel_err(out, ref) <= 1e-6
    R = _R(ref.shape, 13)
    (out * R.to(DEV)).sum().backward()
    (ref * R).sum().backward()
    torch.cuda.synchronize()
    assert tg.grad.dtype == torch.float64
    assert rel_err(Ug.grad, Ur.grad) <= 1e-5
    assert rel_err(tg.grad, tr.grad) <= 1e-5
