"""fp32 error envelope: how far an fp32 implementation of the step may sit
from the exact (float64) result.

For each golden config the oracle runs the step on CPU in float64 and in
fp32 (the reference's own arithmetic: the same aten ops,
nn/network/base.py:141-151), the fp32 run repeated with every fp32 weight
perturbed by at most one ulp (ENSEMBLE runs, fixed seeds): a different but
equally honest rounding of the same step.  The largest distance of those fp32
runs to the float64 result is the error an honest fp32 implementation makes
(for the 64x64 UNet it is dominated by max-pool / ReLU decisions that one-ulp
changes flip); the HIP step is judged against the float64 result with a bar
of ENVELOPE_K times that distance, plus a small floor for quantities whose
fp32 error happens to vanish.  The oracle here is the checker only (test
infrastructure).
"""
import functools

import numpy as np
import torch

from helpers import load_golden, golden_weights, rel_err
from oracle import physics_oracle as O

ENVELOPE_K = 3.0
ENSEMBLE = 10       # one-ulp weight perturbations of the fp32 run (mnist: 2-3 of 10 flip a max-pool/ReLU decision)
# normwise floor: a quantity whose fp32-vs-fp64 error is ~0 (a sum of a few
# exact terms) still gets a few fp32 ulps of room for a different summation order
ENVELOPE_FLOOR = 2e-6
OUT_KEYS = ("enc_pos", "enc_masks", "recons_out", "output_seq", "pos_vel_seq")


def _record(out, L, g):
    d = {k: out[k].detach().double().numpy() for k in OUT_KEYS}
    d.update({"loss_" + k: float(v.detach()) for k, v in L.items()})
    d.update({"grad/" + k: v.detach().double().numpy() for k, v in g.items()})
    return d


def _ulp_perturbed(state, seed):
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, v in state.items():
        if v.dtype == torch.float32:
            u = (torch.rand(v.shape, generator=g, dtype=torch.float64) - 0.5) * 2.0 ** -22   # |u| <= 2^-23
            v = (v.double() * (1 + u)).float()
        out[k] = v
    return out


@functools.lru_cache(maxsize=None)
def oracle_runs(name):
    """(fp64 result, [fp32 result, fp32 results on one-ulp-perturbed weights])."""
    torch.set_num_threads(8)
    z = load_golden(name)
    cfg, _ = O.cfg_from_golden(z)
    state = golden_weights(z)
    x = O.input_from_u8(z["input_u8"])
    f64 = _record(*O.train_step_f64(state, cfg, x))
    f32 = [_record(*O.train_step(state, cfg, x))]
    f32 += [_record(*O.train_step(_ulp_perturbed(state, s), cfg, x)) for s in range(ENSEMBLE)]
    return f64, f32


def oracle_pair(name):
    """(unperturbed fp32 result, fp64 result)."""
    f64, f32 = oracle_runs(name)
    return f32[0], f64


def hip_step(name, conv_math, device):
    """The HIP step on the golden weights/inputs: {key: float64 numpy}."""
    from test_gpu_parity import _model, _input
    z = load_golden(name)
    m = _model(z, device)
    m.conv_math = conv_math
    x = _input(z, device)
    m.output = m(x)
    train_loss, (pred, extrap, recons) = m.compute_loss()
    m.zero_grad(set_to_none=True)
    train_loss.backward()
    torch.cuda.synchronize()
    d = {"enc_pos": m.enc_pos, "enc_masks": m.enc_masks, "recons_out": m.recons_out,
         "output_seq": m.output, "pos_vel_seq": m.pos_vel_seq}
    d = {k: v.detach().double().cpu().numpy() for k, v in d.items()}
    d["loss_train"] = float(train_loss.detach())
    d["loss_extrap"] = float(extrap.detach())
    d["loss_recons"] = float(recons.detach())
    for k, p in m.named_parameters():
        if p.grad is not None:
            d["grad/" + k] = p.grad.detach().double().cpu().numpy()
    return d


def envelope(name, conv_math, device):
    """{key: (hip_err, fp32_err, bar)}: errors normwise-relative to float64;
    fp32_err is the largest over the fp32 ensemble."""
    f64, f32 = oracle_runs(name)
    hip = hip_step(name, conv_math, device)
    rows = {}
    for k in f64:
        if k == "loss_pred":
            continue
        e_hip = rel_err(np.asarray(hip[k]), np.asarray(f64[k]))
        e_32 = max(rel_err(np.asarray(r[k]), np.asarray(f64[k])) for r in f32)
        rows[k] = (e_hip, e_32, max(ENVELOPE_K * e_32, ENVELOPE_FLOOR))
    return rows
