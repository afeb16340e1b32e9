"""ORACLE — test infrastructure only, never the product path.

A CPU (PyTorch fp32, autograd) restatement of the reference's PhysicsNet
training step, written as plain functions over a ``{state_dict key: tensor}``
mapping.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the checker / the timed CPU
baseline.  The product path (``paig_reproduction_amd``) never imports it.

Parity pinning: ``tests/test_oracle_golden.py`` checks every function here
against the golden vectors in ``tests/golden/*.npz``, which
``tests/golden/gen_golden.py`` produced by running the reference itself
(``/root/reference``) on CPU.  So the oracle is pinned to the reference.

Every function cites the reference file:line it restates.  Quirks kept on
purpose: Q3 split-size-1 spring/bouncing cells, Q9 fp64
theta/grid, Q13 ReLU on ShallowUNet's last 1x1 conv, Q2 loss aliasing is a
host-side matter (see ``losses``).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

# runners/torch_run_physics.py:49-75 and nn/network/physics_models.py:31-37
TASKS = {
    #  task:              (cell, seq_len, test_seq_len, input_steps, pred_steps, size, coord_units)
    "bouncing_balls": ("bouncing_ode_cell", 12, 30, 4, 6, 32, 8),
    "spring_color": ("spring_ode_cell", 12, 30, 4, 6, 32, 8),
    "spring_color_half": ("spring_ode_cell", 12, 30, 4, 6, 32, 8),
    "3bp_color": ("gravity_ode_cell", 20, 40, 4, 12, 36, 12),
    "mnist_spring_color": ("spring_ode_cell", 12, 30, 3, 7, 64, 8),
}


class Cfg:
    def __init__(self, task, cell, seq_len, input_steps, pred_steps, size, ae=0.0, alt_vel=False):
        self.task, self.cell = task, cell
        self.seq_len, self.input_steps, self.pred_steps = seq_len, input_steps, pred_steps
        self.size = size
        self.coord_units = TASKS[task][6]
        self.n_objs = self.coord_units // 4          # physics_models.py:96
        self.D = self.coord_units // 2
        self.tmpl = size // 2                         # physics_models.py:101
        self.extrap_steps = seq_len - input_steps - pred_steps
        self.Te = input_steps + pred_steps
        self.R = pred_steps + self.extrap_steps
        self.ae, self.alt_vel = ae, alt_vel
        # "fp32": the reference's arithmetic.  "bf16": BASELINE config #2's
        # (the HIP path's conv_math="bf16"): the U-Net convs' and the dense
        # layers' (l1, l2, alt_vel's linear) matrix operands rounded to bf16
        # (round to nearest even) in the forward, the data and the weight
        # gradient, products accumulated in fp32; biases, bias gradients and
        # everything else (softmax, c13's 1x1 head, l3, velocity MLP, physics,
        # decoder) stay fp32 as in the reference.
        self.operands = "fp32"


def _rb(t):
    """fp32 -> bf16 (round to nearest even) -> fp32."""
    return t.to(torch.bfloat16).to(t.dtype)


class _ConvBF16(torch.autograd.Function):
    """conv2d(x, w) + b, 3x3 or 1x1 "same", with bf16-rounded operands in all
    three products (forward, data gradient, weight gradient), fp32 sums."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return F.conv2d(_rb(x), _rb(w), b, padding="same")

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        pad = w.shape[-1] // 2
        dyb = _rb(dy)
        dx = torch.nn.grad.conv2d_input(x.shape, _rb(w), dyb, padding=pad) if ctx.needs_input_grad[0] else None
        dw = torch.nn.grad.conv2d_weight(_rb(x), w.shape, dyb, padding=pad)
        return dx, dw, dy.sum((0, 2, 3))


class _LinearBF16(torch.autograd.Function):
    """x W^T + b with bf16-rounded operands in all three products."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return _rb(x) @ _rb(w).t() + b

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dyb = _rb(dy)
        dx = dyb @ _rb(w) if ctx.needs_input_grad[0] else None
        return dx, dyb.t() @ _rb(x), dy.sum(0)


def _linear(x, w, b, bf16=False):
    return _LinearBF16.apply(x, w, b) if bf16 else F.linear(x, w, b)


def _conv(P, name, x, relu, bf16=False):
    if bf16:
        y = _ConvBF16.apply(x, P[name + ".weight"], P[name + ".bias"])
    else:
        y = F.conv2d(x, P[name + ".weight"], P[name + ".bias"], padding="same")
    return F.relu(y) if relu else y


def _up(x, size):
    # torchvision Resize(BILINEAR) on tensors == bilinear, align_corners=False,
    # antialias=True (a no-op for 2x upsampling); blocks.py:137,148,160,260,269
    return F.interpolate(x, size=(size, size), mode="bilinear", align_corners=False, antialias=True)


def shallow_unet(P, x, p="encoder.shallow_unet", bf16=False):
    """nn/network/blocks.py:278-308 (note: c7/c10 un-ReLU'd, c13 ReLU'd, Q13).
    bf16: c1..c12 with bf16 operands; the 1x1 head c13 in fp32 (the HIP
    path's fused mask-softmax head computes it in fp32 FMAs)."""
    W = x.shape[-1]

    def conv(name, h_, relu):
        return _conv(P, name, h_, relu, bf16 and not name.endswith(".c13"))

    h = conv(p + ".c1", x, True)
    x1 = conv(p + ".c2", h, True)
    h = F.max_pool2d(x1, 2)
    h = conv(p + ".c3", h, True)
    x2 = conv(p + ".c4", h, True)
    h = F.max_pool2d(x2, 2)
    h = conv(p + ".c5", h, True)
    h = conv(p + ".c6", h, True)
    h = conv(p + ".c7", _up(h, W // 2), False)
    h = torch.cat([h, x2], 1)
    h = conv(p + ".c8", h, True)
    h = conv(p + ".c9", h, True)
    h = conv(p + ".c10", _up(h, W), False)
    h = torch.cat([h, x1], 1)
    h = conv(p + ".c11", h, True)
    h = conv(p + ".c12", h, True)
    return conv(p + ".c13", h, True)


def unet(P, x, p="encoder.unet", bf16=False):
    """nn/network/blocks.py:172-237 (upsamp=True; c9/c12/c15/c18 un-ReLU'd)."""
    W = x.shape[-1]

    def conv(name, h_, relu):
        return _conv(P, name, h_, relu, bf16 and not name.endswith(".c18"))

    h = conv(p + ".c1", x, True)
    x1 = conv(p + ".c2", h, True)
    h = conv(p + ".c3", F.max_pool2d(x1, 2), True)
    x2 = conv(p + ".c4", h, True)
    h = conv(p + ".c5", F.max_pool2d(x2, 2), True)
    x3 = conv(p + ".c6", h, True)
    h = conv(p + ".c7", F.max_pool2d(x3, 2), True)
    h = conv(p + ".c8", h, True)
    h = conv(p + ".c9", _up(h, W // 4), False)
    h = torch.cat([h, x3], 1)
    h = conv(p + ".c10", h, True)
    h = conv(p + ".c11", h, True)
    h = conv(p + ".c12", _up(h, W // 2), False)
    h = torch.cat([h, x2], 1)
    h = conv(p + ".c13", h, True)
    h = conv(p + ".c14", h, True)
    h = conv(p + ".c15", _up(h, W), False)
    h = torch.cat([h, x1], 1)
    h = conv(p + ".c16", h, True)
    h = conv(p + ".c17", h, True)
    return conv(p + ".c18", h, False)


def encoder(P, cfg, frames):
    """ConvolutionalEncoder.forward, nn/network/blocks.py:77-103.
    frames [N,C,H,W] -> enc_pos [N, 2K], enc_masks [N, K+1, H, W], masked objs list."""
    K, H = cfg.n_objs, cfg.size
    bf = getattr(cfg, "operands", "fp32") == "bf16"
    logits = shallow_unet(P, frames, bf16=bf) if H < 40 else unet(P, frames, bf16=bf)
    logits = torch.cat([logits, torch.ones_like(logits[:, :1])], 1)
    masks = torch.softmax(logits, dim=1)
    objs = [masks[:, i:i + 1] * frames for i in range(K)]
    h = torch.cat(objs, 0)
    if H >= 40:
        h = F.avg_pool2d(h, 2)
    h = h.reshape(h.shape[0], -1)
    h = F.relu(_linear(h, P["encoder.l1.weight"], P["encoder.l1.bias"], bf))
    h = F.relu(_linear(h, P["encoder.l2.weight"], P["encoder.l2.bias"], bf))
    h = F.linear(h, P["encoder.l3.weight"], P["encoder.l3.bias"])
    h = torch.cat(torch.split(h, h.shape[0] // K, 0), 1)
    return torch.tanh(h) * (H / 2) + H / 2, masks, objs


def vfn(P, name, shape):
    """VariableFromNetwork.forward, nn/network/blocks.py:318-322 (ones[1,10] input)."""
    x = torch.ones(1, 10)
    x = torch.tanh(F.linear(x, P[name + ".l1.weight"], P[name + ".l1.bias"]))
    return F.linear(x, P[name + ".l2.weight"], P[name + ".l2.bias"]).reshape(shape)


def decoder_sources(P, cfg):
    """The step-constant decoder inputs (physics_models.py:163-171,185-186, Q12)."""
    K, h, H = cfg.n_objs, cfg.tmpl, cfg.size
    template = vfn(P, "var_net_template", [K, 1, h, h])
    contents = vfn(P, "var_net_content", [K, 3, h, h])
    bg = torch.sigmoid(vfn(P, "var_net_background", [1, 3, H, H]))
    joint = torch.cat([template.repeat(1, 3, 1, 1) + 5, torch.sigmoid(contents)], 1)
    return joint, bg


def st_decoder(cfg, joint, bg, pos):
    """conv_st_decoder, nn/network/physics_models.py:151-199 + stn, nn/network/stn.py:5-16.
    pos [N, 2K] -> frames [N, 3, H, W].  theta/grid in float64 (Q9)."""
    K, h, H = cfg.n_objs, cfg.tmpl, cfg.size
    N = pos.shape[0]
    outs = []
    for k in range(K):
        loc = pos[:, 2 * k:2 * k + 2]
        one = torch.ones(N, dtype=torch.float64)
        zero = torch.zeros(N, dtype=torch.float64)
        t2 = ((H / 2 - loc[:, 0]) / h).double()
        t5 = ((H / 2 - loc[:, 1]) / h).double()
        theta = torch.stack([one, zero, t2, zero, one, t5], 1).view(-1, 2, 3)
        grid = F.affine_grid(theta, [N, 6, H, H], align_corners=False)
        src = joint[k:k + 1].expand(N, -1, -1, -1)
        o = F.grid_sample(src, grid.to(src.dtype), mode="bilinear", padding_mode="zeros", align_corners=False)
        outs.append((o[:, :3], o[:, 3:]))
    masks = torch.stack([t - 5 for t, _ in outs] + [torch.ones_like(outs[0][0])], 1)
    masks = torch.softmax(masks, 1)
    conts = [c for _, c in outs] + [bg.expand(N, -1, -1, -1)]
    return sum(masks[:, i] * conts[i] for i in range(K + 1))


def st_decoder_parts(cfg, joint, bg, pos):
    """transf_contents / transf_masks of conv_st_decoder
    (nn/network/physics_models.py:186-196): K warped contents + the tiled
    background, and the K+1 softmax masks, each [N, 3, H, W]."""
    K, h, H = cfg.n_objs, cfg.tmpl, cfg.size
    N = pos.shape[0]
    outs = []
    for k in range(K):
        loc = pos[:, 2 * k:2 * k + 2]
        one = torch.ones(N, dtype=torch.float64)
        zero = torch.zeros(N, dtype=torch.float64)
        t2 = ((H / 2 - loc[:, 0]) / h).double()
        t5 = ((H / 2 - loc[:, 1]) / h).double()
        theta = torch.stack([one, zero, t2, zero, one, t5], 1).view(-1, 2, 3)
        grid = F.affine_grid(theta, [N, 6, H, H], align_corners=False)
        o = F.grid_sample(joint[k:k + 1].expand(N, -1, -1, -1), grid.to(joint.dtype), mode="bilinear",
                          padding_mode="zeros", align_corners=False)
        outs.append((o[:, :3], o[:, 3:]))
    contents = [c for _, c in outs] + [bg.expand(N, -1, -1, -1)]
    masks = torch.softmax(torch.stack([t - 5 for t, _ in outs] + [torch.ones_like(outs[0][0])], 1), 1)
    return contents, torch.unbind(masks, 1)


def velocity_encoder(P, cfg, pos_in):
    """VelocityEncoder.forward, nn/network/blocks.py:31-49.  pos_in [B, in, D] -> [B, D]."""
    K, ins = cfg.n_objs, cfg.input_steps
    if cfg.alt_vel:
        d = pos_in[:, 1:] - pos_in[:, :-1]
        h = torch.cat(torch.chunk(d, K, dim=2), 0).reshape(K * pos_in.shape[0], (ins - 1) * 2)
        h = _linear(h, P["velocity_encoder.init_vel_linear.weight"], P["velocity_encoder.init_vel_linear.bias"],
                    getattr(cfg, "operands", "fp32") == "bf16")
    else:
        h = torch.cat(torch.chunk(pos_in, K, dim=2), 0).reshape(K * pos_in.shape[0], ins * 2)
        pfx = "velocity_encoder.init_vel_mlp."
        h = torch.tanh(F.linear(h, P[pfx + "0.weight"], P[pfx + "0.bias"]))
        h = torch.tanh(F.linear(h, P[pfx + "2.weight"], P[pfx + "2.bias"]))
        h = F.linear(h, P[pfx + "4.weight"], P[pfx + "4.bias"])
    return torch.cat(torch.chunk(h, K, 0), 1)


def spring_cell(P, pos, vel):
    """spring_ode_cell.forward, nn/network/cells.py:31-51 (split size 1: Q3)."""
    dt, k, eq = P["rollout_cell.dt"], P["rollout_cell.k"], P["rollout_cell.equil"]
    p = list(torch.split(pos, 1, 1))
    v = list(torch.split(vel, 1, 1))
    for _ in range(5):
        n = torch.sqrt(torch.abs(torch.sum((p[0] - p[1]) ** 2, dim=-1, keepdim=True)))
        d = (p[0] - p[1]) / (n + 1e-4)
        Fs = torch.exp(k) * (n - 2 * torch.exp(eq)) * d
        v[0] = v[0] - dt / 5 * Fs
        v[1] = v[1] + dt / 5 * Fs
        p[0] = p[0] + dt / 5 * v[0]
        p[1] = p[1] + dt / 5 * v[1]
    return torch.cat(p, 1), torch.cat(v, 1)


def bouncing_cell(P, pos, vel):
    """bouncing_ode_cell.forward, nn/network/cells.py:60-83 (split size 1: Q3)."""
    dt = P["rollout_cell.dt"]
    p = list(torch.split(pos, 1, 1))
    v = list(torch.split(vel, 1, 1))
    for _ in range(5):
        p[0] = p[0] + dt / 5 * v[0]
        p[1] = p[1] + dt / 5 * v[1]
        for j in range(2):
            v[j] = torch.where(p[j] + 2 > 32, -v[j], v[j])
            v[j] = torch.where(0.0 > p[j] - 2, -v[j], v[j])
            p[j] = torch.where(p[j] + 2 > 32, 32 - (p[j] + 2 - 32) - 2, p[j])
            p[j] = torch.where(0.0 > p[j] - 2, -(p[j] - 2) + 2, p[j])
    return torch.cat(p, 1), torch.cat(v, 1)


def gravity_cell(P, pos, vel):
    """gravity_ode_cell.forward, nn/network/cells.py:96-106; A recomputed per call (Q4)."""
    dt = P["rollout_cell.dt"]
    A = torch.exp(P["rollout_cell.g"]) * torch.exp(2 * P["rollout_cell.m"])
    for _ in range(5):
        vecs = [pos[:, 0:2] - pos[:, 2:4], pos[:, 2:4] - pos[:, 4:6], pos[:, 4:6] - pos[:, 0:2]]
        norms = [torch.sqrt(torch.clamp(torch.sum(v ** 2, dim=-1, keepdim=True), min=1e-1, max=1e5)) for v in vecs]
        Fs = [v / torch.pow(torch.clamp(n, min=1, max=170), 3) for v, n in zip(vecs, norms)]
        Fs = [Fs[0] - Fs[2], Fs[1] - Fs[0], Fs[2] - Fs[1]]
        Fs = torch.cat([-A * f for f in Fs], 1)
        vel = vel + dt / 5 * Fs
        pos = pos + dt / 5 * vel
    return pos, vel


CELLS = {"spring_ode_cell": spring_cell, "bouncing_ode_cell": bouncing_cell, "gravity_ode_cell": gravity_cell}


def forward(P, cfg, x):
    """PhysicsNet.conv_feedforward, nn/network/physics_models.py:204-245.
    x [B,T,C,H,W] -> dict of the attributes the reference sets."""
    B, H = x.shape[0], cfg.size
    Te, D = cfg.Te, cfg.D
    h = x[:, :Te].reshape(B * Te, 3, H, H)
    enc_pos, masks, objs = encoder(P, cfg, h)
    joint, bg = decoder_sources(P, cfg)
    recons = st_decoder(cfg, joint, bg, enc_pos).reshape(B, Te, 3, H, H)
    enc_pos = enc_pos.reshape(B, Te, D)
    if cfg.input_steps > 1:
        vel = velocity_encoder(P, cfg, enc_pos[:, :cfg.input_steps])
    else:
        vel = torch.zeros(B, D)
    pos = enc_pos[:, cfg.input_steps - 1]
    cell = CELLS[cfg.cell]
    pv, outs = [torch.cat([pos, vel], 1)], []
    for _ in range(cfg.R):
        pos, vel = cell(P, pos, vel)
        outs.append(st_decoder(cfg, joint, bg, pos))
        pv.append(torch.cat([pos, vel], 1))
    return {
        "enc_pos": enc_pos, "enc_masks": masks, "masked_objs": objs, "recons_out": recons,
        "output_seq": torch.stack(outs, 1), "pos_vel_seq": torch.stack(pv, 1),
    }


def losses(cfg, x, out):
    """PhysicsNet.compute_loss, nn/network/physics_models.py:119-142.
    Returns the TRUE pred loss; the reference's in-place ``+=`` (Q2) makes its
    logged pred_loss equal train_loss, which callers emulate if they need to."""
    rl = torch.sum(torch.square(x[:, :cfg.Te] - out["recons_out"]), dim=[2, 3, 4]).mean()
    L = torch.sum(torch.square(x[:, cfg.input_steps:] - out["output_seq"]), dim=[2, 3, 4])
    pred = L[:, :cfg.pred_steps].mean()
    extrap = L[:, cfg.pred_steps:].mean()
    train = pred + cfg.ae * rl if cfg.ae > 0.0 else pred
    return {"train": train, "pred": pred, "extrap": extrap, "recons": rl}


LIVE_EXCLUDE = ("encoder.unet.", "rollout_cell.weight_", "rollout_cell.bias_")


def live_params(state, cfg):
    """Params that receive a gradient in fresh mode (Q8 dead weights excluded)."""
    dead = "encoder.unet." if cfg.size < 40 else "encoder.shallow_unet."
    out = {}
    for k, v in state.items():
        if k.startswith(dead) or k.startswith("rollout_cell.weight_") or k.startswith("rollout_cell.bias_"):
            continue
        if k in ("rollout_cell.dt", "rollout_cell.m"):
            continue
        if cfg.cell == "bouncing_ode_cell" and k in ("rollout_cell.k", "rollout_cell.equil"):
            continue
        out[k] = v
    return out


def train_step(state, cfg, x, with_grads=True):
    """One fresh-mode step: forward, losses, backward (nn/network/base.py:141-151).
    state: dict key -> tensor (CPU).  Returns (out, losses, grads)."""
    P = {k: (v.detach().clone().requires_grad_(True) if k in live_params(state, cfg) else v.detach())
         for k, v in state.items()}
    out = forward(P, cfg, x)
    L = losses(cfg, x, out)
    grads = {}
    if with_grads:
        L["train"].backward()
        grads = {k: P[k].grad for k in live_params(state, cfg) if P[k].grad is not None}
    return out, L, grads


def train_step_f64(state, cfg, x, with_grads=True):
    """The same step in float64 throughout (state, input, constants, grid):
    the envelope against which fp32 implementations are judged."""
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return train_step({k: v.double() for k, v in state.items()}, cfg, x.double(), with_grads)
    finally:
        torch.set_default_dtype(prev)


def train_trajectory(state, cfg, xs, lr, steps, f64=False):
    """``steps`` fresh-mode steps with torch.optim.RMSprop semantics
    (nn/network/base.py:141-152, :14 defaults), batch xs[s % len(xs)].
    Returns (per-step [train, pred(aliased: = train, Q2), extrap, recons],
    final state).  f64: the whole loop in float64 (the envelope)."""
    prev = torch.get_default_dtype()
    if f64:
        torch.set_default_dtype(torch.float64)
        state = {k: v.double() for k, v in state.items()}
        xs = [x.double() for x in xs]
    try:
        state = {k: v.detach().clone() for k, v in state.items()}
        live = live_params(state, cfg)
        sq = {k: torch.zeros_like(state[k]) for k in live}
        losses = []
        for s in range(steps):
            x = xs[s % len(xs)]
            out, L, grads = train_step(state, cfg, x)
            t = float(L["train"].detach())
            losses.append([t, t, float(L["extrap"].detach()), float(L["recons"].detach())])
            with torch.no_grad():
                for k, g in grads.items():
                    rmsprop_step(state[k], g, sq[k], lr)
        return losses, state
    finally:
        torch.set_default_dtype(prev)


def reference_mode_steps(state, cfg, x_eval, xs, lr):
    """The reference's ACTUAL training step (quirk Q1, nn/network/base.py:141-143
    vs :195): ``self.output`` is the last eval forward's (no grad); each train
    step's loss reads it for pred/extrap while the gradient reaches only the
    current forward's reconstruction term (encoder + decoder sources; the
    rollout, velocity MLP and physics parameters get None and RMSprop skips
    them).  Returns (per-step losses, first step's grads, final state)."""
    state = {k: v.detach().clone() for k, v in state.items()}
    live = live_params(state, cfg)
    sq = {k: torch.zeros_like(state[k]) for k in live}
    with torch.no_grad():
        stale = forward(state, cfg, x_eval)["output_seq"]
    losses, g0 = [], None
    for x in xs:
        P = {k: (v.requires_grad_(True) if k in live else v) for k, v in state.items()}
        out = forward(P, cfg, x)
        rl = torch.sum(torch.square(x[:, :cfg.Te] - out["recons_out"]), dim=[2, 3, 4]).mean()
        L = torch.sum(torch.square(x[:, cfg.input_steps:] - stale), dim=[2, 3, 4])
        pred, extrap = L[:, :cfg.pred_steps].mean(), L[:, cfg.pred_steps:].mean()
        train = pred + cfg.ae * rl if cfg.ae > 0.0 else pred
        t = float(train.detach())
        losses.append([t, t, float(extrap), float(rl.detach())])
        train.backward()
        grads = {k: P[k].grad for k in live if P[k].grad is not None}
        if g0 is None:
            g0 = {k: g.clone() for k, g in grads.items()}
        with torch.no_grad():
            for k, g in grads.items():
                rmsprop_step(state[k], g, sq[k], lr)
        state = {k: v.detach() for k, v in state.items()}
    return losses, g0, state


def eval_metrics(state, cfg, x):
    """eval_performance over ONE whole-set batch (Q15), nn/network/base.py:174-211:
    {eval_pred_loss (= train, Q2), eval_extrap_loss, eval_recons_loss} and the outputs."""
    with torch.no_grad():
        out = forward(state, cfg, x)
        L = losses(cfg, x, out)
    return {"eval_pred_loss": float(L["train"]), "eval_extrap_loss": float(L["extrap"]),
            "eval_recons_loss": float(L["recons"])}, out


def rmsprop_step(param, grad, square_avg, lr, alpha=0.99, eps=1e-8):
    """torch.optim.RMSprop defaults (nn/network/base.py:14): in-place update."""
    square_avg.mul_(alpha).addcmul_(grad, grad, value=1 - alpha)
    param.addcdiv_(grad, square_avg.sqrt().add_(eps), value=-lr)


def cfg_from_golden(z):
    task, cell, seq_len, ins, pred, size, B, ae, alt = [str(s) for s in z["config"]]
    return Cfg(task, cell, int(seq_len), int(ins), int(pred), int(size), float(ae), bool(int(alt))), int(B)


def input_from_u8(u8):
    N, T, H, W, C = u8.shape
    return torch.from_numpy((u8.astype(np.float32).reshape(N, T, C, H, W) / 255).astype(np.float32))


_ = math  # keep import (used by callers for pi etc.)
