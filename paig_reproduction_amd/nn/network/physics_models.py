"""PhysicsNet — the reference's model surface (nn/network/physics_models.py:40-330)
on the MI355X-native step.

Same constructor signature/positional order, attributes, state_dict keys and
init RNG stream as the reference, so it is a drop-in for
runners/torch_run_physics.py.  ``forward``/``conv_feedforward`` run the whole
step (encoder U-Net -> localiser -> velocity MLP -> physics rollout -> STN
decoder, fused per-frame SSE) through libpaig_hip.so as ONE autograd node whose
backward is the explicit HIP backward (paig_reproduction_amd.engine).
"""
import inspect
import logging
import os
import weakref

import ctypes

import numpy as np
import torch
import torch.nn as pnn

from paig_reproduction_amd._lib import lib, ptr, stream_handle, require_device
from paig_reproduction_amd.engine import Engine
from paig_reproduction_amd.flat import FlatParams
from paig_reproduction_amd.nn.network.base import OPTIMIZERS, BaseNetTorch
from paig_reproduction_amd.nn.network.blocks import ConvolutionalEncoder, VelocityEncoder, VariableFromNetwork
from paig_reproduction_amd.nn.network.cells import bouncing_ode_cell, spring_ode_cell, gravity_ode_cell

logger = logging.getLogger("tf")

CELLS = {
    "bouncing_ode_cell": bouncing_ode_cell,
    "spring_ode_cell": spring_ode_cell,
    "gravity_ode_cell": gravity_ode_cell,
    "lstm": pnn.LSTMCell,
}

COORD_UNITS = {
    "bouncing_balls": 8,
    "spring_color": 8,
    "spring_color_half": 8,
    "3bp_color": 12,
    "mnist_spring_color": 8,
}


class _PhysicsStep(torch.autograd.Function):
    """The whole forward as one node; backward = engine.backward."""

    @staticmethod
    def forward(ctx, anchor, x, engine):
        need = ctx.needs_input_grad[0]
        res, S = engine.forward(x, need_saved=need)
        ctx.engine = engine
        ctx.S = S
        ctx.set_materialize_grads(False)
        engine.last_masked_objs = res["masked_objs"]
        outs = (res["output_seq"], res["recons_out"], res["enc_pos"], res["pos_vel_seq"], res["sse_rec"],
                res["sse_roll"], res["enc_masks"], res["template"], res["contents"], res["background_content"])
        ctx.mark_non_differentiable(res["enc_masks"], res["template"], res["contents"], res["background_content"])
        return outs

    @staticmethod
    def backward(ctx, d_out, d_rec, d_enc, d_pvs, d_sse_rec, d_sse_roll, *unused):
        if ctx.S is None:
            raise RuntimeError("PhysicsNet step was run without saving activations")
        flat = ctx.engine.model._flat
        acc = flat.begin_backward()
        # the live-steps mark of _LossReduce.backward holds only while the
        # gradient tensor is unmodified: autograd may accumulate a second
        # gradient path into it in place (InputBuffer's add_), which keeps the
        # tensor (and the attribute) but bumps its version counter
        mark = getattr(d_sse_roll, "_paig_live_steps", None) if d_out is None else None
        live = mark[0] if mark is not None and d_sse_roll._version == mark[1] else 0
        # in-kernel loss weights (_LossReduce.backward): only for the unmodified stand-ins
        lw = {}
        for key, g in (("rec", d_sse_rec), ("roll", d_sse_roll)):
            m = getattr(g, "_paig_lossw", None)
            if m is not None and g._version == m[2]:
                lw[key] = m[:2]
        # incoming gradients may be broadcast views (d sum(sse)/d sse is an
        # expanded scalar, stride 0): the kernels read dense vectors
        d_sse_rec = d_sse_rec.contiguous() if d_sse_rec is not None else None
        d_sse_roll = d_sse_roll.contiguous() if d_sse_roll is not None else None
        ctx.engine.backward(ctx.S, d_sse_rec, d_sse_roll, d_out, d_rec, d_enc, d_pvs, roll_live=live, lossw=lw)
        # nothing reached the rollout branch (quirk Q1: the loss read a stale
        # output): the velocity encoder and physics parameters are not in the
        # graph, so like torch they get grad None (their flat slots hold zeros)
        none = ctx.engine.model.ROLLOUT_PARAMS if d_out is None and d_sse_roll is None and d_pvs is None else ()
        flat.end_backward(acc, none)
        ctx.S = None
        return None, None, None


_LOSSW = {}


def _lossw_buffers(dev, n_rec, n_roll):
    """Persistent NaN-filled stand-ins for the loss-weight gradients (one pair
    per device and size; filled once, outside any graph capture: the first
    training steps run eagerly)."""
    key = (str(dev), n_rec, n_roll)
    if key not in _LOSSW:
        _LOSSW[key] = (torch.full((n_rec,), float("nan"), device=dev), torch.full((n_roll,), float("nan"), device=dev))
    return _LOSSW[key]


class _LossReduce(torch.autograd.Function):
    """Per-frame SSE -> (train, extrap, recons) (physics_models.py:119-141):
    train = pred + ae * recons formed in the kernel -- the value the
    reference's in-place ``+=`` leaves in BOTH train_loss and pred_loss (Q2)."""

    @staticmethod
    def forward(ctx, sse_rec, sse_roll, B, Te, R, pred, ae):
        dev = sse_rec.device
        o = [torch.empty((), device=dev) for _ in range(3)]
        lib().paig_loss_reduce(ptr(sse_rec), ptr(sse_roll), B, Te, R, pred, float(ae), ptr(o[0]), ptr(o[1]),
                               ptr(o[2]), stream_handle(dev))
        ctx.shape = (B, Te, R, pred, float(ae))
        ctx.dev = dev
        ctx.set_materialize_grads(False)
        return o[0], o[1], o[2]

    @staticmethod
    def backward(ctx, dt, de, dr):
        B, Te, R, pred, ae = ctx.shape
        if os.environ.get("PAIG_LOSSW_INKERNEL", "1") != "0" and not torch.is_grad_enabled():
            # the per-frame weights are formed inside the decoder backwards
            # from these adjoints (paig_decoder_bwd_ex lw modes): the returned
            # gradients are persistent NaN buffers carrying the adjoints, so a
            # path that reads them as values (another gradient accumulated into
            # them) gets NaN, never silent garbage
            wrec, wroll = _lossw_buffers(ctx.dev, B * Te, B * R)
            lw = (dt, de, dr, ae, B, Te, R, pred)
            wrec._paig_lossw = (1, lw, wrec._version)
            wroll._paig_lossw = (2, lw, wroll._version)
            if de is None:
                wroll._paig_live_steps = (pred, wroll._version)
            return wrec, wroll, None, None, None, None, None
        wrec = torch.empty(B * Te, device=ctx.dev)
        wroll = torch.empty(B * R, device=ctx.dev)
        lib().paig_loss_bwd(ptr(dt), ptr(de), ptr(dr), ae, ptr(wrec), ptr(wroll), B, Te, R, pred,
                            stream_handle(ctx.dev))
        if de is None:
            # no extrapolation loss in the graph: only the first pred steps of
            # every sequence carry a weight (physics_models.py:129-139), so the
            # rollout decoder backward walks those frames only.  The mark
            # carries the tensor's version: a gradient that autograd
            # accumulates with another one (in place or not) no longer
            # matches it and falls back to every frame.
            wroll._paig_live_steps = (pred, wroll._version)
        return wrec, wroll, None, None, None, None, None


class _FrameSSE(torch.autograd.Function):
    """Per-frame SSE of dense frames vs input[:, ins:] (the unfused path, for a
    loss on frames that are not the current forward's, e.g. quirk Q1)."""

    @staticmethod
    def forward(ctx, frames, x, ins):
        B, R = frames.shape[0], frames.shape[1]
        T = x.shape[1]
        if x.shape[0] != B or tuple(x.shape[2:]) != tuple(frames.shape[2:]) or T - ins != R:
            # the reference's (input[:, ins:] - output) would not broadcast either
            raise RuntimeError(f"compute_loss: output {tuple(frames.shape)} does not match input[:, {ins}:] of "
                               f"{tuple(x.shape)}")
        fr = 3 * frames.shape[-1] * frames.shape[-2]
        frames = frames.contiguous()
        x = x.contiguous()
        sse = torch.empty(B * R, device=frames.device)
        lib().paig_frame_sse(ptr(frames), fr, 0, 0, ptr(x) + ins * fr * 4, T * fr, R, fr, ptr(sse), B * R, fr,
                             stream_handle(frames.device))
        ctx.save_for_backward(frames, x)
        ctx.meta = (ins, B, R, T, fr)
        return sse

    @staticmethod
    def backward(ctx, w):
        frames, x = ctx.saved_tensors
        ins, B, R, T, fr = ctx.meta
        d = torch.empty_like(frames)
        lib().paig_frame_sse_bwd(ptr(frames), fr, 0, 0, ptr(x) + ins * fr * 4, T * fr, R, fr, ptr(w.contiguous()),
                                 ptr(d), B * R, fr, stream_handle(frames.device))
        return d, None, None


class PhysicsNet(BaseNetTorch):
    def __init__(self,
                 task="",
                 recurrent_units=128,
                 lstm_layers=1,
                 cell_type="",
                 seq_len=20,
                 input_steps=3,
                 pred_steps=5,
                 autoencoder_loss=0.0,
                 alt_vel=False,
                 color=False,
                 input_size=36 * 36,
                 encoder_type="",
                 decoder_type="conv_st_decoder",
                 device=torch.device("cpu")):
        super().__init__()
        self.device = device
        assert task in COORD_UNITS
        self.task = task
        self.recurrent_units = recurrent_units
        self.lstm_layers = lstm_layers
        self.cell_type = cell_type
        self.cell = CELLS[self.cell_type]
        if self.cell is pnn.LSTMCell:
            raise NotImplementedError("the 'lstm' black-box cell cannot be called by the reference's rollout "
                                      "(physics_models.py:233 signature mismatch); not supported")
        self.color = color
        self.conv_ch = 3 if color else 1
        if not color:
            # Q11: the template is tiled to 3 channels regardless of --color, so
            # grayscale breaks in the reference too.
            raise ValueError("PhysicsNet requires color=True (reference quirk Q11: grayscale is broken)")
        self.input_size = input_size
        self.conv_input_shape = [self.conv_ch] + [int(np.sqrt(input_size))] * 2
        self.input_shape = [self.conv_ch] + [int(np.sqrt(input_size))] * 2
        self.decoder = {name: method for name, method in
                        inspect.getmembers(self, predicate=inspect.ismethod) if "decoder" in name}[decoder_type]
        self.output_shape = self.conv_input_shape
        assert seq_len > input_steps + pred_steps
        assert input_steps >= 1
        assert pred_steps >= 1
        self.seq_len = seq_len
        self.input_steps = input_steps
        self.pred_steps = pred_steps
        self.extrap_steps = self.seq_len - self.input_steps - self.pred_steps
        self.alt_vel = alt_vel
        self.autoencoder_loss = autoencoder_loss
        self.coord_units = COORD_UNITS[self.task]
        self.n_objs = self.coord_units // 4
        self.extra_valid_fns.append((self.visualize_sequence, [], {}))
        self.extra_test_fns.append((self.visualize_sequence, [], {}))
        tmpl_size = self.conv_input_shape[1] // 2
        self.log_sig = 1.
        if self.log_sig != 1.:
            raise NotImplementedError("sigma != 1")
        # Network subcomponents (creation order = reference order, for init parity)
        self.var_net_content = VariableFromNetwork([self.n_objs, self.conv_ch, tmpl_size, tmpl_size])
        self.var_net_background = VariableFromNetwork([1, *self.input_shape])
        self.var_net_template = VariableFromNetwork([self.n_objs, 1, tmpl_size, tmpl_size])
        self.encoder = ConvolutionalEncoder(self.conv_input_shape, 200, 2, self.n_objs, self.device)
        self.velocity_encoder = VelocityEncoder(self.alt_vel, self.input_steps, self.n_objs, self.coord_units,
                                                self.device)
        self.rollout_cell = self.cell(self.coord_units // 2, self.coord_units // 2)
        # the standalone U-Net / encoder forwards run on this model's engine
        for mod in (self.encoder, self.encoder.shallow_unet, self.encoder.unet):
            object.__setattr__(mod, "_paig_owner", weakref.ref(self))
        object.__setattr__(self, "_parts", None)
        self.loss_mode = "fresh"
        # conv arithmetic of the HIP path: "split" (fp32-accurate split-precision
        # 16-bit MFMA, default), "fp32" (f32-input MFMA) or "bf16"
        self.conv_math = os.environ.get("PAIG_CONV_MATH", "split")
        self._init_native()

    # ------------------------------------------------------------ native ----
    # gradients final before the U-Net backward starts (VariableFromNetwork and
    # the localiser's l1/l2: ~97% of the gradient bytes) lead the flat buffer,
    # so their data-parallel all-reduce can start while the U-Net backward runs
    EARLY_GRADS = ("var_net_content.", "var_net_background.", "var_net_template.", "encoder.l1.", "encoder.l2.")
    # parameters reached only through the rollout branch
    ROLLOUT_PARAMS = ("velocity_encoder.", "rollout_cell.")

    def _live_names(self):
        dead = "encoder.unet." if self.conv_input_shape[1] < 40 else "encoder.shallow_unet."
        names = []
        for n, p in self.named_parameters():
            if n.startswith(dead) or n.startswith("rollout_cell."):
                continue
            names.append(n)
        names = ([n for n in names if n.startswith(self.EARLY_GRADS)] +
                 [n for n in names if not n.startswith(self.EARLY_GRADS)])
        if self.cell_type == "spring_ode_cell":
            names += ["rollout_cell.k", "rollout_cell.equil"]
        elif self.cell_type == "gravity_ode_cell":
            names += ["rollout_cell.g"]
        return names

    def _init_native(self):
        object.__setattr__(self, "_flat", FlatParams(self, self._live_names(), early=self.EARLY_GRADS))
        object.__setattr__(self, "_engine", None)
        object.__setattr__(self, "_anchor", None)

    @property
    def _param_by_name(self):
        return dict(self.named_parameters())

    def _native(self):
        if self._engine is None:
            object.__setattr__(self, "_engine", Engine(self))
        self._flat.ensure()
        if self._anchor is None:
            object.__setattr__(self, "_anchor", torch.zeros((), requires_grad=True))
        return self._engine

    # ------------------------------------------------------------- API ----
    def get_batch(self, batch_size, iterator):
        batch_x, _ = iterator.next_batch(batch_size)
        feed_dict = {"input": batch_x}
        return feed_dict, (batch_x, None)

    def compute_loss(self):
        """nn/network/physics_models.py:119-142, including the in-place ``+=``
        that makes pred_loss alias train_loss (Q2)."""
        B, Te, R = self.input.shape[0], self.input_steps + self.pred_steps, self.pred_steps + self.extrap_steps
        sse_rec = self._sse_rec
        if self.output is self._fwd_output:
            sse_roll = self._sse_roll
        else:
            sse_roll = _FrameSSE.apply(self.output, self.input, self.input_steps)
        # train = pred + ae * recons in one kernel; pred_loss IS train_loss, as
        # after the reference's in-place ``train_loss += ae * recons`` (Q2)
        train, extrap, recons = _LossReduce.apply(sse_rec, sse_roll, B, Te, R, self.pred_steps,
                                                  self.autoencoder_loss)
        self.recons_loss = recons
        self.pred_loss = train
        self.extrap_loss = extrap
        train_loss = self.pred_loss
        eval_losses = [self.pred_loss, self.extrap_loss, self.recons_loss]
        return train_loss, eval_losses

    def build_optimizer(self, base_lr, optimizer="rmsprop", anneal_lr=True):
        self.base_lr = base_lr
        self.anneal_lr = anneal_lr
        self.lr = base_lr
        self._flat.ensure()
        self.optimizer = OPTIMIZERS[optimizer](self, self.lr)

    def conv_st_decoder(self, inp):
        """Decode positions [N, coord_units/2] -> frames [N, C, H, W]
        (physics_models.py:151-199): the three VariableFromNetwork sources and
        the HIP STN/compositing decoder, differentiable w.r.t. the positions and
        the sources' parameters.  Sets template / contents / background_content
        like the reference; transf_contents / transf_masks are formed on request."""
        require_device(inp)
        from paig_reproduction_amd.nn.network.native_modules import _STDecoder
        self._native()
        out = _STDecoder.apply(inp, self._anchor_for_modules(), self)
        srcs = self._last_sources
        K, H = self.n_objs, self.conv_input_shape[1]
        h = H // 2
        self.template = srcs["tmpl"].view(K, 1, h, h)
        self.contents = srcs["cont"].view(K, 3, h, h)
        self.background_content = srcs["bg"].view(1, 3, H, H)
        object.__setattr__(self, "_parts", (inp.detach().float().contiguous(), 2 * K, srcs))
        return out

    def check_numerics(self):
        """Raise if a split-precision kernel flagged an operand outside f16's
        range since the last check.  The step's operands (activations,
        gradients, weights) are all scaled by powers of two from their own
        maxima and have no range limit; the flag remains for the fixed-scale
        fallbacks of the C ABI (a conv weight gradient called without the
        forward's xmax slots, GEMM math 1 / 5), which the step never takes.
        Synchronises the device: BaseNetTorch calls it at log steps only."""
        if self.conv_math != "split":
            return
        rc = lib().paig_f16_range_status(1)
        if rc != 0:
            raise FloatingPointError(
                "split-precision path: an operand beyond the f16 staging range of a fixed-scale fallback "
                "kernel; rerun with --conv_math fp32" if rc > 0 else f"paig_f16_range_status failed ({rc})")

    def _anchor_for_modules(self):
        return torch.zeros((), requires_grad=True)

    _VFN_SRCS = (("var_net_template", "tmpl", 0), ("var_net_content", "cont", 0), ("var_net_background", "bg", 1))

    def _decoder_sources(self, dev, st):
        """The decoder's step-constant sources (physics_models.py:163-171,
        185-186): raw template, raw contents, sigmoid(background)."""
        L = lib()
        K, H = self.n_objs, self.conv_input_shape[1]
        h = H // 2
        sizes = {"tmpl": K * h * h, "cont": K * 3 * h * h, "bg": 3 * H * H}
        pd = self._param_by_name
        srcs = {}
        for nm, key, post in self._VFN_SRCS:
            P = sizes[key]
            srcs[nm] = (torch.empty(200, device=dev), torch.empty(P, device=dev),
                        torch.empty(P, device=dev) if post else None, P)
        arr = lambda xs: (ctypes.c_void_p * 3)(*xs)   # noqa: E731
        L.paig_vfn_fwd_multi(3, *[arr([ptr(pd[nm + suf]) for nm, _, _ in self._VFN_SRCS])
                                  for suf in (".l1.weight", ".l1.bias", ".l2.weight", ".l2.bias")],
                             arr([ptr(srcs[nm][0]) for nm, _, _ in self._VFN_SRCS]),
                             arr([ptr(srcs[nm][1]) for nm, _, _ in self._VFN_SRCS]),
                             arr([ptr(srcs[nm][2]) for nm, _, _ in self._VFN_SRCS]),
                             (ctypes.c_int * 3)(*[srcs[nm][3] for nm, _, _ in self._VFN_SRCS]), st)
        out = {"tmpl": srcs["var_net_template"][1], "cont": srcs["var_net_content"][1],
               "bg": srcs["var_net_background"][2], "_vfn": srcs}
        object.__setattr__(self, "_last_sources", out)
        return out

    def _decoder_sources_backward(self, srcs, dsrc, st):
        """dsrc = [d template | d sigmoid(content) | d sigmoid(background)] (the
        decoder's source gradients) -> the three VariableFromNetworks' parameter
        gradients, deposited into the flat gradient buffer."""
        from paig_reproduction_amd.flat import deposit_grad
        L = lib()
        dev = dsrc.device
        v = srcs["_vfn"]
        pd = self._param_by_name
        offs, o = [], 0
        for nm, _, _ in self._VFN_SRCS:
            offs.append(o)
            o += v[nm][3]
        g = {nm: {suf: torch.empty_like(pd[nm + suf]) for suf in (".l1.weight", ".l1.bias", ".l2.weight", ".l2.bias")}
             for nm, _, _ in self._VFN_SRCS}
        parts = [torch.empty(L.paig_vfn_bwd_blocks(v[nm][3]) * 200, device=dev) for nm, _, _ in self._VFN_SRCS]
        arr = lambda xs: (ctypes.c_void_p * 3)(*xs)   # noqa: E731
        # content and background enter through a sigmoid (sig = 1)
        L.paig_vfn_bwd_multi(3, arr([ptr(dsrc) + 4 * off for off in offs]),
                             arr([ptr(v[nm][1]) for nm, _, _ in self._VFN_SRCS]), (ctypes.c_int * 3)(0, 1, 1),
                             arr([ptr(v[nm][0]) for nm, _, _ in self._VFN_SRCS]),
                             arr([ptr(pd[nm + ".l2.weight"]) for nm, _, _ in self._VFN_SRCS]),
                             *[arr([ptr(g[nm][suf]) for nm, _, _ in self._VFN_SRCS])
                               for suf in (".l1.weight", ".l1.bias", ".l2.weight", ".l2.bias")],
                             arr([ptr(pt) for pt in parts]), (ctypes.c_int * 3)(*[v[nm][3] for nm, _, _ in self._VFN_SRCS]),
                             st)
        for nm, _, _ in self._VFN_SRCS:
            for suf, t in g[nm].items():
                deposit_grad(pd[nm + suf], t)

    def _transf_parts(self):
        """(transf_contents, transf_masks) of the last decoder call
        (physics_models.py:186-196): K warped contents + the tiled background,
        and the K+1 compositing masks, each [N, 3, H, W] (detached)."""
        if self._parts is None:
            raise AttributeError("transf_contents / transf_masks: no decoder call yet")
        cached = getattr(self, "_parts_cache", None)
        if cached is not None and cached[0] is self._parts:
            return cached[1]
        pos, inner, srcs = self._parts
        K, H = self.n_objs, self.conv_input_shape[1]
        N = pos.shape[0]
        dev = pos.device
        cont = torch.empty(K + 1, N, 3, H, H, device=dev)
        masks = torch.empty(K + 1, N, 3, H, H, device=dev)
        lib().paig_decoder_parts(ptr(pos), inner, ptr(srcs["tmpl"]), ptr(srcs["cont"]), ptr(srcs["bg"]), ptr(cont),
                                 ptr(masks), N, K, H // 2, H, stream_handle(dev))
        res = ([cont[k] for k in range(K + 1)], tuple(masks[k] for k in range(K + 1)))
        object.__setattr__(self, "_parts_cache", (self._parts, res))
        return res

    @property
    def transf_contents(self):
        return self._transf_parts()[0]

    @property
    def transf_masks(self):
        return self._transf_parts()[1]

    def forward(self, input):
        return self.conv_feedforward(input)

    def conv_feedforward(self, inp):
        """nn/network/physics_models.py:204-245 as one fused native step."""
        require_device(inp)
        eng = self._native()
        self.input = inp
        x = inp.detach()
        if x.dtype != torch.float32:
            x = x.float()
        outs = _PhysicsStep.apply(self._anchor, x, eng)
        (out, recons, enc_pos, pvs, sse_rec, sse_roll, masks, tmpl, cont, bg) = outs
        self.recons_out = recons
        self.enc_pos = enc_pos
        self.pos_vel_seq = pvs
        self.enc_masks = masks
        self.masked_objs = eng.last_masked_objs
        self.template, self.contents, self.background_content = tmpl, cont, bg
        self._sse_rec, self._sse_roll = sse_rec, sse_roll
        # the reference's last decoder call decodes the last rollout step
        R, D = self.pred_steps + self.extrap_steps, self.coord_units // 2
        object.__setattr__(self, "_parts", (pvs.detach()[:, R, :D], (R + 1) * 2 * D,
                                            {"tmpl": tmpl.detach(), "cont": cont.detach(), "bg": bg.detach()}))
        self._fwd_output = out
        return out

    def visualize_sequence(self):
        """physics_models.py:247-330, reduced to what this image supports:
        example%d.jpg grids and extra_outputs.npz (the gif needs moviepy,
        absent here).  Off the hot path."""
        try:
            import matplotlib
            matplotlib.use("agg")
            import matplotlib.pyplot as plt
        except Exception:  # pragma: no cover
            return
        batch_size = min(self.batch_size, 4)
        feed_dict, (batch_x, _) = self.get_batch(batch_size, self.test_iterator)
        if torch.is_tensor(batch_x):   # device-resident dataset (F2)
            batch_x = batch_x.detach().cpu().numpy()
        if not hasattr(self, "output") or self.output is None:
            return
        output_seq = self.output.detach().cpu().numpy()[:batch_size]
        recons_seq = self.recons_out.detach().cpu().numpy()[:batch_size]
        n = min(batch_size, output_seq.shape[0], batch_x.shape[0])
        for i in range(n):
            seq = np.concatenate([batch_x[i, :self.input_steps], output_seq[i]], 0)
            rows = [seq, batch_x[i], np.concatenate([recons_seq[i], np.zeros(
                (self.extrap_steps,) + recons_seq.shape[2:], dtype=recons_seq.dtype)], 0)]
            grid = np.concatenate([np.concatenate(list(r.reshape(r.shape[0], *self.input_shape[1:],
                                                                 self.conv_ch)), 1) for r in rows], 0)
            fig, ax = plt.subplots(figsize=(grid.shape[1] // 32, grid.shape[0] // 32 + 1))
            ax.imshow(np.clip(grid, 0, 1), interpolation="nearest")
            ax.axis("off")
            fig.savefig(os.path.join(self.save_dir, "example%d.jpg" % i))
            plt.close(fig)
        np.savez_compressed(os.path.join(self.save_dir, "extra_outputs.npz"),
                            contents=self.contents.detach().cpu().numpy(),
                            templates=self.template.detach().cpu().numpy(),
                            background_content=self.background_content.detach().cpu().numpy(),
                            enc_masks=self.enc_masks.detach().cpu().numpy())
