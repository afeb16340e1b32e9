"""Standalone, differentiable forwards of PhysicsNet's submodules on the HIP
kernels (the reference's module surface, nn/network/blocks.py,
nn/network/cells.py, nn/network/stn.py, callable one at a time):

  VariableFromNetwork()        blocks.py:318-322   paig_vfn_fwd / paig_vfn_bwd
  VelocityEncoder(inp)         blocks.py:31-49     paig_velmlp_* / paig_vel_pack + paig_gemm_ex
  <cell>(poss, vels)           cells.py:31-106     paig_rollout_fwd/bwd with R = 1
  ShallowUNet / UNet (x)       blocks.py:278-308 / :172-237   the engine's U-Net plan
  ConvolutionalEncoder (inp)   blocks.py:77-103    the engine's encoder stage
  PhysicsNet.conv_st_decoder   physics_models.py:151-199      paig_vfn_* + paig_decoder_*
  stn(U, theta, out_size)      stn.py:5-16         paig_stn_fwd/bwd

The training step does not use these: it runs the whole step fused
(engine.Engine).  They exist so a caller of the reference's modules finds
them working; each is one torch.autograd.Function whose backward calls the
backward kernels and deposits parameter gradients with torch semantics into
the model's flat gradient buffer (flat.deposit_grad / partial_backward), so
FlatOptimizer and the data-parallel all-reduce see them.  Gradients flow to
the inputs that require them.  Nothing falls back to torch math.
"""
import ctypes

import torch

from paig_reproduction_amd._lib import lib, ptr, stream_handle, require_device
from paig_reproduction_amd.flat import deposit_grad


def _anchor():
    return torch.zeros((), requires_grad=True)


def _f32(t):
    require_device(t)
    return t.detach().float().contiguous()


# ----------------------------------------------------------- VFN ----------
class _VFN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, mod):
        W1, b1, W2, b2 = mod.l1.weight, mod.l1.bias, mod.l2.weight, mod.l2.bias
        require_device(W1)
        dev = W1.device
        P = W2.shape[0]
        h, y = torch.empty(200, device=dev), torch.empty(P, device=dev)
        lib().paig_vfn_fwd(ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(h), ptr(y), None, P, stream_handle(dev))
        ctx.mod, ctx.h, ctx.y = mod, h, y
        return y

    @staticmethod
    def backward(ctx, dy):
        mod, h, y = ctx.mod, ctx.h, ctx.y
        dev, P = y.device, y.numel()
        L = lib()
        g = {"W1": torch.empty(200, 10, device=dev), "b1": torch.empty(200, device=dev),
             "W2": torch.empty(P, 200, device=dev), "b2": torch.empty(P, device=dev)}
        part = torch.empty(L.paig_vfn_bwd_blocks(P) * 200, device=dev)
        L.paig_vfn_bwd(ptr(dy.float().contiguous()), ptr(y), 0, ptr(h), ptr(mod.l2.weight), ptr(g["W1"]),
                       ptr(g["b1"]), ptr(g["W2"]), ptr(g["b2"]), ptr(part), P, stream_handle(dev))
        for p, k in ((mod.l1.weight, "W1"), (mod.l1.bias, "b1"), (mod.l2.weight, "W2"), (mod.l2.bias, "b2")):
            deposit_grad(p, g[k])
        return None, None


def vfn_forward(mod):
    """VariableFromNetwork.forward(): l2(tanh(l1(ones[1, 10]))) reshaped to mod.shape."""
    return _VFN.apply(_anchor(), mod).view(*[int(s) for s in mod.shape])


# ----------------------------------------------------------- cells --------
class _Cell(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pos, vel, anchor, cell):
        pos, vel = _f32(pos), _f32(vel)
        B, D = pos.shape
        assert vel.shape == (B, D), (tuple(vel.shape), (B, D))
        dev = pos.device
        kind = cell.KIND
        p0, p1 = _cell_params(cell)
        pvs = torch.empty(B, 2, 2 * D, device=dev)
        # the kernel takes the initial velocity in the velocity encoder's
        # row layout [n_objs][B][2] (a relayout copy of [B][2 n_objs])
        vk = vel.view(B, D // 2, 2).permute(1, 0, 2).contiguous()
        lib().paig_rollout_fwd(kind, ptr(pos), D, ptr(vk), ptr(cell.dt), ptr(p0), ptr(p1), ptr(pvs), B, D, 1,
                               stream_handle(dev))
        ctx.cell, ctx.pvs = cell, pvs
        return pvs[:, 1, :D].clone(), pvs[:, 1, D:].clone()

    @staticmethod
    def backward(ctx, dpos1, dvel1):
        cell, pvs = ctx.cell, ctx.pvs
        B, _, D2 = pvs.shape
        D = D2 // 2
        dev = pvs.device
        L = lib()
        dpvs = torch.zeros(B, 2, 2 * D, device=dev)
        if dpos1 is not None:
            dpvs[:, 1, :D] = dpos1
        if dvel1 is not None:
            dpvs[:, 1, D:] = dvel1
        dpos_roll = torch.zeros(B, 1, D, device=dev)
        dpos0, dvel0 = torch.empty(B, D, device=dev), torch.empty(B, D, device=dev)
        part = torch.empty(2 * L.paig_rollout_bwd_blocks(B), device=dev, dtype=torch.float64)
        gq = torch.zeros(2, device=dev, dtype=torch.float64)
        p0, p1 = _cell_params(cell)
        L.paig_rollout_bwd(cell.KIND, ptr(pvs), ptr(dpos_roll), ptr(dpvs), ptr(cell.dt), ptr(p0), ptr(p1), ptr(dpos0),
                           ptr(dvel0), ptr(part), ptr(gq), ptr(gq) + 8, 0, B, D, 1, stream_handle(dev))
        if cell.KIND == 0:
            deposit_grad(cell.k, gq[0])
            deposit_grad(cell.equil, gq[1])
        elif cell.KIND == 2:
            deposit_grad(cell.g, gq[0])
        # dvel0 comes back in the [n_objs][B][2] layout
        return dpos0, dvel0.view(D // 2, B, 2).permute(1, 0, 2).reshape(B, D), None, None


def _cell_params(cell):
    if cell.KIND == 0:
        return cell.k, cell.equil
    if cell.KIND == 2:
        return cell.g, cell.m
    return None, None


def cell_forward(cell, poss, vels):
    """<cell>.forward(poss, vels): 5 substeps (cells.py:31-51 / 60-83 / 96-106)."""
    return _Cell.apply(poss, vels, _anchor(), cell)


# ----------------------------------------------------------- velocity -----
class _VelEnc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inp, anchor, mod):
        inp = _f32(inp)
        B, S, D = inp.shape
        K = mod.n_objs
        assert S == mod.input_steps and D == 2 * K, (tuple(inp.shape), mod.input_steps, K)
        dev = inp.device
        st = stream_handle(dev)
        L = lib()
        vel = torch.empty(B, D, device=dev)
        if mod.alt_vel:
            X = torch.empty(K * B, 2 * (S - 1), device=dev)
            L.paig_vel_pack(ptr(inp), ptr(X), B, S, K, S, 1, st)
            W, b = mod.init_vel_linear.weight, mod.init_vel_linear.bias
            y = torch.empty(K * B, 2, device=dev)
            L.paig_gemm_ex(0, 1, K * B, 2, 2 * (S - 1), 1.0, ptr(X), 2 * (S - 1), ptr(W), 2 * (S - 1), 0.0, ptr(y), 2,
                           ptr(b), 0, 0, None, 0, None, None, 0, 0, st)
            ctx.saved = (X,)
            # rows k*B + b -> vel[b][2k + j] (torch.chunk / cat, blocks.py:40-41): a relayout copy
            vel = y.view(K, B, 2).permute(1, 0, 2).reshape(B, D)
        else:
            pm = mod.init_vel_mlp
            X = torch.empty(K * B, 2 * S, device=dev)
            h1, h2 = torch.empty(K * B, 100, device=dev), torch.empty(K * B, 100, device=dev)
            vk = torch.empty(K * B, 2, device=dev)   # rows k*B + b, as the fused path keeps it
            L.paig_velmlp_fwd(ptr(inp), B, S, K, S, ptr(pm[0].weight), ptr(pm[0].bias), ptr(pm[2].weight),
                              ptr(pm[2].bias), ptr(pm[4].weight), ptr(pm[4].bias), ptr(X), ptr(h1), ptr(h2), ptr(vk),
                              st)
            vel = vk.view(K, B, 2).permute(1, 0, 2).reshape(B, D)   # torch.chunk / cat (blocks.py:47-48)
            ctx.saved = (X, h1, h2)
        ctx.mod, ctx.shape = mod, (B, S, D, K)
        return vel

    @staticmethod
    def backward(ctx, dvel):
        mod = ctx.mod
        B, S, D, K = ctx.shape
        dev = dvel.device
        st = stream_handle(dev)
        L = lib()
        dvel = dvel.float().contiguous()
        dinp = torch.zeros(B, S, D, device=dev)
        if mod.alt_vel:
            (X,) = ctx.saved
            dy = dvel.view(B, K, 2).permute(1, 0, 2).contiguous()   # [K*B][2] (relayout)
            W = mod.init_vel_linear.weight
            gW, gb = torch.empty_like(W), torch.empty(2, device=dev)
            dX = torch.empty_like(X)
            n = X.shape[1]
            L.paig_gemm_ex(1, 0, 2, n, K * B, 1.0, ptr(dy), 2, ptr(X), n, 0.0, ptr(gW), n, None, 0, 0, None, 0,
                           ptr(gb), None, 0, 0, st)
            L.paig_gemm_ex(0, 0, K * B, n, 2, 1.0, ptr(dy), 2, ptr(W), n, 0.0, ptr(dX), n, None, 0, 0, None, 0, None,
                           None, 0, 0, st)
            deposit_grad(W, gW)
            deposit_grad(mod.init_vel_linear.bias, gb)
            L.paig_vel_unpack_add(ptr(dX), None, ptr(dinp), B, S, K, S, 1, st)
        else:
            X, h1, h2 = ctx.saved
            dvel = dvel.view(B, K, 2).permute(1, 0, 2).contiguous()   # back to rows k*B + b
            pm = mod.init_vel_mlp
            rows = K * B
            nblk, slen = L.paig_velmlp_bwd_blocks(rows), L.paig_velmlp_slab_len(S)
            slab = torch.empty(nblk * slen, device=dev)
            dX = torch.empty_like(X)
            L.paig_velmlp_bwd(ptr(dvel), ptr(X), ptr(h1), ptr(h2), ptr(pm[0].weight), ptr(pm[2].weight),
                              ptr(pm[4].weight), ptr(dX), ptr(slab), rows, S, st)
            g = torch.empty(slen, device=dev)
            L.paig_slab_reduce(ptr(slab), nblk, slen, slen, ptr(g), 0, st)
            o = 0
            for p in (pm[0].weight, pm[0].bias, pm[2].weight, pm[2].bias, pm[4].weight, pm[4].bias):
                deposit_grad(p, g[o:o + p.numel()])
                o += p.numel()
            L.paig_vel_unpack_add(ptr(dX), None, ptr(dinp), B, S, K, S, 0, st)
        return dinp, None, None


def velocity_forward(mod, inp):
    """VelocityEncoder.forward(inp [B, input_steps, coord_units/2]) -> [B, coord_units/2]."""
    return _VelEnc.apply(inp, _anchor(), mod)


# ----------------------------------------------------------- STN ----------
class _STN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, U, theta, out_size):
        # a float64 theta keeps its precision for the grid (affine_grid in
        # theta's dtype, cast to fp32 before sampling: stn.py:12-14)
        f64 = theta.dtype == torch.float64
        U = _f32(U)
        require_device(theta)
        th = theta.detach().reshape(-1, 6).to(torch.float64 if f64 else torch.float32).contiguous()
        N, C, Hi, Wi = U.shape
        assert th.shape[0] == N, ("stn: U and theta batch differ", N, th.shape[0])
        Ho, Wo = int(out_size[0]), int(out_size[1])
        out = torch.empty(N, C, Ho, Wo, device=U.device)
        fwd = lib().paig_stn_fwd_f64 if f64 else lib().paig_stn_fwd
        fwd(ptr(U), ptr(th), ptr(out), N, C, Hi, Wi, Ho, Wo, stream_handle(U.device))
        ctx.save_for_backward(U, th)
        ctx.tshape = theta.shape
        ctx.dtypes = (theta.dtype,)
        return out

    @staticmethod
    def backward(ctx, dout):
        U, th = ctx.saved_tensors
        N, C, Hi, Wi = U.shape
        Ho, Wo = dout.shape[-2:]
        dU = torch.zeros_like(U) if ctx.needs_input_grad[0] else None
        dth = torch.empty_like(th) if ctx.needs_input_grad[1] else None
        bwd = lib().paig_stn_bwd_f64 if th.dtype == torch.float64 else lib().paig_stn_bwd
        bwd(ptr(U), ptr(th), ptr(dout.float().contiguous()), ptr(dU), ptr(dth), N, C, Hi, Wi, Ho, Wo,
            stream_handle(U.device))
        if dth is not None:
            dth = dth.view(ctx.tshape).to(ctx.dtypes[0])
        return dU, dth, None


def stn(U, theta, out_size):
    """stn.py:5-16: affine_grid(theta.view(-1, 2, 3)) + grid_sample (bilinear,
    zeros, align_corners=False) of U [N, C, Hi, Wi] to out_size (Ho, Wo)."""
    return _STN.apply(U, theta, tuple(out_size))


def batch_transformer(U, thetas, out_size):
    """stn.py:18-23: U [N, C, H, W] repeated for each of thetas' [N, T, 6] transforms."""
    num_batch, num_transforms = thetas.shape[:2]
    rep = U.unsqueeze(1).expand(num_batch, num_transforms, *U.shape[1:]).reshape(-1, *U.shape[1:])
    return stn(rep, thetas, out_size)


# ----------------------------------------------------------- decoder ------
class _STDecoder(torch.autograd.Function):
    """conv_st_decoder (physics_models.py:151-199) with its three
    VariableFromNetwork sources: positions [N, 2K] -> frames [N, 3, H, W]."""

    @staticmethod
    def forward(ctx, pos, anchor, model):
        pos = _f32(pos)
        dev = pos.device
        st = stream_handle(dev)
        L = lib()
        K, H = model.n_objs, model.conv_input_shape[1]
        h = H // 2
        N = pos.shape[0]
        srcs = model._decoder_sources(dev, st)
        out = torch.empty(N, 3, H, H, device=dev)
        L.paig_decoder_fwd(ptr(pos), 0, 2 * K, 0, ptr(srcs["tmpl"]), ptr(srcs["cont"]), ptr(srcs["bg"]), ptr(out),
                           3 * H * H, None, 0, 0, 0, None, N, K, h, H, st)
        ctx.model, ctx.pos, ctx.srcs = model, pos, srcs
        return out

    @staticmethod
    def backward(ctx, dout):
        model, pos, srcs = ctx.model, ctx.pos, ctx.srcs
        dev = pos.device
        st = stream_handle(dev)
        L = lib()
        K, H = model.n_objs, model.conv_input_shape[1]
        h = H // 2
        N = pos.shape[0]
        dout = dout.float().contiguous()
        slab_len = int(L.paig_decoder_slab_len(K, h, H))
        nb = L.paig_decoder_bwd_blocks(N, 0, 0, K, h, H)
        slab = torch.empty(nb * slab_len, device=dev)
        scr_n = L.paig_decoder_bwd_scratch(N, K, h, H)
        scratch = torch.empty(scr_n, device=dev) if scr_n else None
        dpos = torch.empty(N, 2 * K, device=dev)
        # no target frames: the SSE weight is null and dL/dout comes dense
        # (the target pointer must still address N valid frames; dout does)
        L.paig_decoder_bwd(ptr(pos), 0, 2 * K, 0, ptr(srcs["tmpl"]), ptr(srcs["cont"]), ptr(srcs["bg"]), ptr(dout),
                           3 * H * H, 0, 0, None, ptr(dout), 3 * H * H, ptr(dpos), ptr(slab), ptr(scratch), N, 0, K, h, H,
                           st)
        dsrc = torch.empty(slab_len, device=dev)
        L.paig_slab_reduce(ptr(slab), nb, slab_len, slab_len, ptr(dsrc), 0, st)
        model._decoder_sources_backward(srcs, dsrc, st)
        return dpos, None, None


# ----------------------------------------------------------- encoder ------
class _Encoder(torch.autograd.Function):
    """ConvolutionalEncoder.forward (which="encoder") or the U-Net alone
    (which="unet" / "shallow_unet") over independent frames [N, 3, H, W],
    on the fused step's own stages (engine._encoder_forward / _unet_forward
    and their backward).  No gradient w.r.t. the frames themselves (the
    reference never uses it, Q10); masks / masked objects are outputs only."""

    @staticmethod
    def forward(ctx, x, anchor, model, which, need_saved=True):
        from paig_reproduction_amd.engine import Layout, _empty
        x = _f32(x)
        N = x.shape[0]
        H = model.conv_input_shape[1]
        assert tuple(x.shape[1:]) == (3, H, H), (tuple(x.shape), H)
        eng = model._native()
        net = "unet" if which == "unet" else ("shallow_unet" if which == "shallow_unet" else None)
        lay = Layout(model, N, 1, frames=N, net=net)
        dev = x.device
        st = stream_handle(dev)
        ws = _empty(eng.workspace_floats(lay), dev)
        # need_saved False (no autograd graph): the U-Net workspace without
        # gradient buffers, slabs or pool codes (PAIG_UNET_INFERENCE)
        S = {"lay": lay, "x": x, "ws": ws, "dev": dev, "cm": eng.conv_flags(), "need_saved": need_saved}
        x_view = (ptr(x), lay.frame, 0, 0)
        ctx.model, ctx.S, ctx.which = model, S, which
        if which == "encoder":
            eng._encoder_forward(S, lay, x_view, ws, st)
            K, HW = lay.K, lay.HW
            masks = S["masks"].view(N, K + 1, H, H)
            objs = S["objs"].view(K, N, 3, H, H)
            ctx.mark_non_differentiable(masks, objs)
            return S["enc_pos"].view(N, 2 * K), masks, objs
        S["x_view"] = x_view
        eng._unet_forward(S, lay, x_view, st)
        return S["acts"]["LG"].view(N, lay.K, H, H).clone()

    @staticmethod
    def backward(ctx, *grads):
        model, S, which = ctx.model, ctx.S, ctx.which
        eng = model._native()
        lay = S["lay"]
        st = stream_handle(S["dev"])
        if which == "encoder":
            denc = grads[0]
            if denc is None:
                return None, None, None, None, None
            with model._flat.partial_backward(("encoder.",)):
                eng._encoder_backward(S, denc.float().contiguous(), st, hook=False)
        else:
            # (paig_unet_bwd_ex applies ShallowUNet c13's ReLU' itself, Q13)
            dLG = grads[0].float().contiguous()
            with model._flat.partial_backward((lay.prefix,)):
                eng._unet_backward(S, dLG, st)
        return None, None, None, None, None


def encoder_forward(enc, inp):
    """ConvolutionalEncoder.forward(inp) -> (enc_pos [N, 2K], enc_masks, masked_objs list)."""
    model = _owner(enc)
    pos, masks, objs = _Encoder.apply(inp, model._anchor_for_modules(), model, "encoder", _need_saved(model))
    return pos, masks, [objs[k] for k in range(objs.shape[0])]


def unet_forward(unet, x, which):
    """ShallowUNet / UNet forward(x) -> logits [N, n_objs, H, W]."""
    model = _owner(unet)
    return _Encoder.apply(x, model._anchor_for_modules(), model, which, _need_saved(model))


def _need_saved(model):
    """Whether a backward can follow (grad mode on, some parameter trainable):
    else the forward allocates no training workspace."""
    return torch.is_grad_enabled() and any(q.requires_grad for q in model.parameters())


def _owner(mod):
    ref = getattr(mod, "_paig_owner", None)
    model = ref() if ref is not None else None
    if model is None:
        raise RuntimeError(f"{type(mod).__name__}: the HIP forward runs on the PhysicsNet that owns this module "
                           "(its flat parameter buffer and engine); construct it through PhysicsNet")
    return model
