"""Native PhysicsNet step: forward and backward of the reference's training
path, every FLOP in libpaig_hip.so (include/paig_hip.h), orchestrated here.

Reference path: PhysicsNet.conv_feedforward
(nn/network/physics_models.py:204-245) -> compute_loss (:119-142) ->
loss.backward() -> optimizer.step() (nn/network/base.py:141-152).

What is different from the reference, by design (results are the same):
  * the decoder runs ONCE over all B*(Te+R) frames instead of R+1 calls;
    the per-frame SSE of the loss is fused into it;
  * VariableFromNetwork outputs are computed once per step (Q12);
  * the backward is explicit (no autograd graph of ~2k aten nodes): the
    whole step is one autograd.Function whose backward calls the kernels in
    reverse order, writing parameter gradients straight into one flat
    gradient buffer (ready for a single RCCL all-reduce and a fused
    optimizer kernel);
  * the 5-substep physics rollout is one kernel for all R steps.
Nothing here falls back to PyTorch math: torch is used only for device
memory (caching allocator), streams and the autograd hook.
"""
import ctypes
import os

import torch

from ._lib import PaigError, lib, ptr, stream_handle, require_device

# The U-Net plans (ShallowUNet blocks.py:240-308, UNet :106-237: buffers,
# ops, which upsamples / pools fuse into which convs, the backward's
# write / accumulate / ReLU' bookkeeping) live in ONE place: csrc/unet.hip,
# whose C-ABI interpreter (paig_unet_fwd_ex / paig_unet_bwd_ex) IS the
# engine's U-Net stage.  Python only names the convs (c1..cN, plan order).


class Layout:
    """Static shapes of one step (from the PhysicsNet config and batch)."""

    def __init__(self, model, B, T, frames=None, net=None):
        """frames=N: the encoder alone over N independent frames (the
        standalone ConvolutionalEncoder / U-Net calls): F = N, no sequence.
        net: "unet" / "shallow_unet" to plan that U-Net whatever the frame
        size (both are built, Q8; the live one is chosen by H otherwise)."""
        self.B, self.T = B, T
        self.K = model.n_objs
        self.D = model.coord_units // 2
        self.H = model.conv_input_shape[1]
        self.h = self.H // 2
        self.ins, self.pred = model.input_steps, model.pred_steps
        self.Te = self.ins + self.pred
        self.R = model.pred_steps + model.extrap_steps
        if frames is None:
            assert T == model.seq_len, f"input has {T} frames, model expects seq_len={model.seq_len}"
            self.F = B * self.Te
        else:
            self.F = frames
        self.alt_vel = model.alt_vel
        self.cell = {"spring_ode_cell": 0, "bouncing_ode_cell": 1, "gravity_ode_cell": 2}[model.cell_type]
        self.unet = self.H >= 40 if net is None else net == "unet"
        L = lib()
        self.net = 1 if self.unet else 0   # paig_unet_*: 0 ShallowUNet(hidden 8), 1 UNet(hidden 16)
        self.prefix = "encoder.unet." if self.unet else "encoder.shallow_unet."
        self.nconv = L.paig_unet_query(self.net, self.K, 0)
        self.lg_relu = not self.unet   # ShallowUNet's c13 output is ReLU'd (Q13), UNet's c18 not
        # l1 input: the masked objects, AvgPool2d(2)'d first for H >= 40 (blocks.py:92-96)
        self.l1_in = 3 * (self.H // 2) ** 2 if self.unet else 3 * self.H * self.H
        self.HW = self.H * self.H
        self.frame = 3 * self.HW
        # the U-Net's last layer, a 1x1 head (ShallowUNet c13, 8 -> K, ReLU'd;
        # UNet c18, 16 -> K, with the objects' AvgPool2d), is fused into the
        # mask softmax (paig_head_mask_fwd_ex / _bwd_ex) in the encoder; the
        # standalone U-Net call keeps it as a conv (its logits are the output).
        # PAIG_FUSE_HEAD=0: the separate conv + softmax kernels (A/B)
        self.head_buf = L.paig_unet_query(self.net, self.K, 2)
        self.head_ci = L.paig_unet_query(self.net, self.K, 3)
        self.head_name = f"c{self.nconv}"
        self.head_flags = (1 if self.lg_relu else 0) | (2 if self.unet else 0)
        self.fuse_head = (self.K in (2, 3) and self.HW % 4 == 0 and os.environ.get("PAIG_FUSE_HEAD", "1") != "0" and
                          ((not self.unet and self.head_ci == 8) or (self.unet and self.head_ci == 16 and
                                                                     self.H % 4 == 0)))
        if self.fuse_head:
            # the fused head kernels read the head input (and write its
            # gradient) as [F][head_ci][H][W] from the start of its buffer
            off, cbuf = L.paig_unet_query(self.net, self.K, 5), L.paig_unet_query(self.net, self.K, 6)
            if off != 0 or cbuf != self.head_ci:
                raise PaigError(f"U-Net head input at channel offset {off} of a {cbuf}-channel buffer: the fused "
                                f"head needs the whole buffer ({self.head_ci} channels from offset 0)")


class KernelProbe:
    """Times every launch of one tagged kernel (``tag``), or of every tagged
    kernel (``tag=None``), with HIP events recorded on the stream it is
    launched on: the main stream; the side-stream chains are not tagged
    (bench.py's roofline numbers)."""

    backlog_cycles = 1 << 20

    def __init__(self, tag):
        self.tag = tag
        self.events = {}
        self.work = {}

    def wrap(self, tag, flops, nbytes=0):
        probe = self
        want = probe.tag is None or tag == probe.tag

        class _Ctx:
            def __enter__(self):
                if want:
                    self.e0 = torch.cuda.Event(enable_timing=True)
                    self.e1 = torch.cuda.Event(enable_timing=True)
                    # a spin kernel first: the stream is then backlogged when the
                    # start event and the probed kernel are enqueued, so the host's
                    # launch latency between them does not count as kernel time
                    torch.cuda._sleep(probe.backlog_cycles)
                    self.e0.record()
                return self

            def __exit__(self, *exc):
                if want:
                    self.e1.record()
                    probe.events.setdefault(tag, []).append((self.e0, self.e1))
                    probe.work[tag] = (flops, nbytes)
                return False

        return _Ctx()

    def overhead_ms(self, n=20):
        """The event pair's own cost around one dispatch: the same bracket
        (backlogged stream, start event, launch, end event) around a spin
        kernel of zero cycles.  Subtracted from the probed intervals so they
        compare with rocprof's kernel start-to-end durations."""
        pairs = []
        for _ in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(self.backlog_cycles)
            e0.record()
            torch.cuda._sleep(0)
            e1.record()
            pairs.append((e0, e1))
        torch.cuda.synchronize()
        return min(a.elapsed_time(b) for a, b in pairs)

    def summaries(self):
        """{tag: {tag, n, avg_ms, avg_ms_raw, flops, bytes}} (per launch;
        avg_ms net of the event bracket's overhead)."""
        torch.cuda.synchronize()
        ovh = self.overhead_ms() if self.events else 0.0
        out = {}
        for tag, evs in self.events.items():
            ms = [a.elapsed_time(b) for a, b in evs]
            fl, nb = self.work[tag]
            raw = sum(ms) / len(ms)
            out[tag] = {"tag": tag, "n": len(ms), "avg_ms": max(raw - ovh, 1e-6), "avg_ms_raw": raw,
                        "overhead_ms": ovh, "flops": fl, "bytes": nb}
        return out

    def summary(self):
        s = self.summaries()
        return s.get(self.tag) if self.tag is not None else None


class _NoProbe:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NOPROBE = _NoProbe()


def _parr(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


def _iarr(vals):
    return (ctypes.c_int * len(vals))(*vals)


def _empty(n, device, dtype=torch.float32):
    return torch.empty(n, device=device, dtype=dtype)


class Engine:
    """Binds a PhysicsNet's parameters to the HIP kernels."""

    def __init__(self, model):
        self.model = model
        self.L = lib()
        self.probe = None
        self.last_masked_objs = None
        self._side = None   # second stream (see _fork)
        # called once per backward when the early gradient bucket is final
        # (FlatParams.allreduce_early by default; bench.py splits its HIP graph here)
        self.bucket_hook = model._flat.allreduce_early
        # DeviceDataIterator.ByteTargets bound to the step's input buffer: the
        # decoders then read their targets as the dataset's bytes
        self.byte_targets = None

    # conv arithmetic (include/paig_hip.h flags): "split" = f16 hi/lo pieces on
    # the 16-bit matrix cores, operands scaled by powers of two (fp32-accurate:
    # within 3x the fp32 reference's own error, tests/test_gpu_envelope.py),
    # "fp32" = f32-input MFMA, "bf16" = bf16 operands (BASELINE config #2)
    CONV_MATH = {"split": 128, "fp32": 0, "bf16": 256}

    # the same choice for the dense layers (paig_gemm_ex math) per GEMM kind
    # (forward, wgrad, dgrad): f16 pieces, both operands (activations /
    # gradients and the weights) scaled by running powers of two (math 6): no
    # range limit on any operand
    GEMM_MATH = {"split": (6, 6, 6), "fp32": (0, 0, 0), "bf16": (3, 3, 3)}
    FWD, WGRAD, DGRAD = 0, 1, 2

    def gemm_math(self, kind):
        return self.GEMM_MATH[getattr(self.model, "conv_math", "split")][kind]

    def conv_flags(self):
        m = getattr(self.model, "conv_math", "split")
        if m not in self.CONV_MATH:
            raise ValueError(f"conv_math must be one of {sorted(self.CONV_MATH)}, got {m!r}")
        return self.CONV_MATH[m]

    @staticmethod
    def _dec_bytes(n, lay, tb=4):
        """Algorithmic HBM bytes of one decoder forward over n frames: the
        target frames read (fused SSE; tb bytes per value: 4 fp32, 1 for the
        dataset's bytes) and the decoded frames written; positions and the
        step-constant sources (< 100 KB) are negligible."""
        return n * lay.frame * (tb + 4)

    @staticmethod
    def _dec_bwd_bytes(live, n, lay, dense, tb=4):
        """Algorithmic HBM bytes of one decoder backward: the targets of the
        `live` frames that carry a loss weight (+ their dense dL/dout when
        given) read, the position gradients of all n frames and the source
        gradients (one slab_len vector) written.  The partial-gradient slab
        rows are the kernel's own overhead, not algorithmic."""
        return (live * lay.frame * (tb + (4 if dense else 0)) + n * 2 * lay.D * 4
                + (4 * lay.K * lay.h * lay.h + 3 * lay.HW) * 4)

    def _p(self, tag, flops=0, nbytes=0):
        """Probe context of one launch: algorithmic FLOPs and HBM bytes (the
        compulsory operand reads + result writes) for bench.py's roofline."""
        return self.probe.wrap(tag, flops, nbytes) if self.probe is not None else _NOPROBE

    # -- parameter access ------------------------------------------------
    def p(self, name):
        return self.model._param_by_name[name]

    def g(self, name):
        return self.model._flat.grad_view(name)

    # -- small helpers ---------------------------------------------------
    def linear(self, x, rows, name, out, act, st, ws):
        """out[rows, O] = act(x[rows, I] W^T + b) ; W = name.weight [O, I]"""
        W, b = self.p(name + ".weight"), self.p(name + ".bias")
        O, I = W.shape
        with self._p("gemm_fwd:" + name, 2 * rows * O * I, 4 * (rows * I + O * I + rows * O)):
            self.L.paig_gemm_ex(0, 1, rows, O, I, 1.0, ptr(x), I, ptr(W), I, 0.0, ptr(out), O, ptr(b), act, 0, None,
                                0, None, ptr(ws), ws.numel() if ws is not None else 0, self.gemm_math(self.FWD), st)

    def linear_bwd(self, x, dy, rows, name, dx, aux, auxm, st, ws, need_dx=True, defer_epi=False):
        """dW = dy^T x and db = colsum(dy) (one GEMM, fused row sums) ; dx = (dy W) * act'(aux).
        defer_epi: the weight gradient's split-K epilogue rides in the next
        GEMM's launch (paig_gemm_defer_epilogue; the caller flushes)."""
        W = self.p(name + ".weight")
        O, I = W.shape
        gW, gb = self.g(name + ".weight"), self.g(name + ".bias")
        n_ws = ws.numel()
        if defer_epi:
            self.L.paig_gemm_defer_epilogue(1)
        with self._p("gemm_wgrad:" + name, 2 * rows * O * I, 4 * (rows * O + rows * I + O * I + O)):
            self.L.paig_gemm_ex(1, 0, O, I, rows, 1.0, ptr(dy), O, ptr(x), I, 0.0, ptr(gW), I, None, 0, 0, None, 0,
                                ptr(gb), ptr(ws), n_ws, self.gemm_math(self.WGRAD), st)
        if need_dx:
            # dY and W read, dX written (+ the activation read for its derivative)
            with self._p("gemm_dgrad:" + name, 2 * rows * O * I, 4 * (rows * O + O * I + (2 if auxm else 1) * rows * I)):
                self.L.paig_gemm_ex(0, 0, rows, I, O, 1.0, ptr(dy), O, ptr(W), I, 0.0, ptr(dx), I, None, 0, auxm,
                                    ptr(aux), I, None, ptr(ws), n_ws, self.gemm_math(self.DGRAD), st)

    def dense_tail(self):
        """The localiser's l2 + head as fp32 FMA inside the launches around
        them (paig_dense_tail_fwd / paig_head_l2_bwd): in split arithmetic,
        where the 3-MFMA l2 GEMMs were latency-bound launches of their own;
        bf16 keeps its 1-MFMA l2 GEMMs (faster there).  PAIG_DENSE_TAIL=0: A/B."""
        return self.gemm_math(self.FWD) == 6 and os.environ.get("PAIG_DENSE_TAIL", "1") != "0"

    def workspace_floats(self, lay):
        K, F, B = lay.K, lay.F, lay.B
        n1 = lay.l1_in
        need = [self.L.paig_gemm_workspace(K * F, 200, n1), self.L.paig_gemm_workspace(K * F, 200, 200),
                self.L.paig_gemm_workspace(200, n1, K * F), self.L.paig_gemm_workspace(K * F, n1, 200), self.L.paig_gemm_workspace(200, 200, K * F),
                self.L.paig_gemm_workspace(2, 200, K * F), self.L.paig_gemm_workspace(100, 100, K * B),
                # l2's and l1's weight-gradient partials side by side (their epilogues are deferred)
                self.L.paig_gemm_workspace(200, 200, K * F) + self.L.paig_gemm_workspace(200, n1, K * F),
                self.L.paig_gemm_workspace(K * B, 100, 100), 1 << 16,
                self.L.paig_gemm_parts_size(K * F, 200, n1, self.gemm_math(self.FWD))]
        return int(max(need))

    # -- forward ---------------------------------------------------------
    def forward(self, x, need_saved=True):
        require_device(x)
        model = self.model
        model._flat.ensure()
        B, T = x.shape[0], x.shape[1]
        lay = Layout(model, B, T)
        dev = x.device
        st = stream_handle(dev)
        L = self.L
        x = x.contiguous()
        K, F, HW, H, h, D = lay.K, lay.F, lay.HW, lay.H, lay.h, lay.D
        ws = _empty(self.workspace_floats(lay), dev)
        S = {"lay": lay, "x": x, "ws": ws, "dev": dev, "need_saved": need_saved}
        cm = self.conv_flags()
        S["cm"] = cm

        # ---- VariableFromNetwork sources (once per step, Q12): allocated here,
        # computed on the main stream while the side stream runs the velocity
        # MLP + rollout (only the decoders read them)
        src = {}
        vf = (("var_net_template", K * h * h, False), ("var_net_content", K * 3 * h * h, False),
              ("var_net_background", 3 * HW, True))
        for nm, P, post in vf:
            src[nm] = (_empty(200, dev), _empty(P, dev), _empty(P, dev) if post else None)
        S["src"] = src
        tmpl, cont, bgp = src["var_net_template"][1], src["var_net_content"][1], src["var_net_background"][2]

        # ---- encoder over the first Te frames of every sequence (in place)
        x_view = (ptr(x), T * lay.frame, lay.Te, lay.frame)   # frame n = b*Te + t
        # the rollout decoders' targets: x's frames, or (byte targets bound to
        # this input buffer) the dataset rows it was gathered from, as bytes.
        # The reconstruction targets are the encoder's frames, which the
        # gather writes as fp32 in either case: read there (no row lookup)
        bt = self.byte_targets
        if bt is not None and bt.covers(x, lay):
            tb = 1
            tgt_roll = (bt.base + lay.ins * lay.frame, bt.idx_ptr, T * lay.frame, lay.R, lay.frame)
        else:
            tb = 0
            tgt_roll = (ptr(x) + lay.ins * lay.frame * 4, T * lay.frame, lay.R, lay.frame)
        S.update(tb=tb, tgt_roll=tgt_roll)
        self._encoder_forward(S, lay, x_view, ws, st)
        masks, objs, enc_pos = S["masks"], S["objs"], S["enc_pos"]

        # Two independent chains follow the position head: velocity MLP ->
        # physics rollout (one thread per sequence: latency-bound, a few
        # blocks) and VFN sources -> reconstruction decode of all B*Te frames.
        # They run on one stream (see _one_stream); PAIG_SCHED=0 puts the first
        # on a side stream.  Everything a side chain touches is allocated
        # before the fork.
        recons = _empty(F * lay.frame, dev)
        sse_rec = _empty(F, dev)
        vel0 = None
        vel_args = None
        if lay.ins > 1:
            S_in = lay.ins
            cols = 2 * (S_in - 1 if lay.alt_vel else S_in)
            Xv = _empty(K * B * cols, dev)
            vel0 = _empty(K * B * 2, dev)
            if lay.alt_vel:
                S.update(Xv=Xv)
            else:
                v1 = _empty(K * B * 100, dev)
                v2 = _empty(K * B * 100, dev)
                S.update(Xv=Xv, v1=v1, v2=v2)
        S["vel0"] = vel0
        pvs = _empty(B * (lay.R + 1) * 2 * D, dev)
        prm = self.cell_params(lay)
        S["pvs"] = pvs

        def velocity(q):   # velocity encoder, then the physics rollout (all R steps in one launch)
            if vel0 is not None:
                if lay.alt_vel:
                    L.paig_vel_pack(ptr(enc_pos), ptr(S["Xv"]), B, lay.Te, K, lay.ins, 1, q)
                    self.linear(S["Xv"], K * B, "velocity_encoder.init_vel_linear", vel0, 0, q, ws)
                else:   # the whole MLP (packing fused) in one launch
                    pm = "velocity_encoder.init_vel_mlp."
                    L.paig_velmlp_fwd(ptr(enc_pos), B, lay.Te, K, lay.ins, *[ptr(self.p(pm + n)) for n in (
                        "0.weight", "0.bias", "2.weight", "2.bias", "4.weight", "4.bias")], ptr(S["Xv"]),
                        ptr(S["v1"]), ptr(S["v2"]), ptr(vel0), q)
            L.paig_rollout_fwd(lay.cell, ptr(enc_pos) + (lay.ins - 1) * D * 4, lay.Te * D, ptr(vel0), ptr(prm[0]),
                               ptr(prm[1]), ptr(prm[2]), ptr(pvs), B, D, lay.R, q)

        def vfn_src(q):    # VariableFromNetwork sources
            L.paig_vfn_fwd_multi(3, *[_parr([ptr(self.p(nm + suf)) for nm, _, _ in vf])
                                      for suf in (".l1.weight", ".l1.bias", ".l2.weight", ".l2.bias")],
                                 _parr([ptr(src[nm][0]) for nm, _, _ in vf]),
                                 _parr([ptr(src[nm][1]) for nm, _, _ in vf]),
                                 _parr([ptr(src[nm][2]) for nm, _, _ in vf]), _iarr([P for _, P, _ in vf]), q)

        def dec_rec(q):    # reconstruction decode (all B*Te frames, SSE vs input fused)
            with self._p("dec_fwd:recon", 0, self._dec_bytes(F, lay)):
                L.paig_decoder_fwd(ptr(enc_pos), 0, 2 * K, 0, ptr(tmpl), ptr(cont), ptr(bgp), ptr(recons),
                                   lay.frame, *x_view, ptr(sse_rec), F, K, h, H, q)

        if self._one_stream():
            if vel0 is not None and not lay.alt_vel and os.environ.get("PAIG_FUSE_VFN", "1") != "0":
                # velocity MLP + VFN sources in one launch (independent), then the rollout
                pm = "velocity_encoder.init_vel_mlp."
                L.paig_velmlp_vfn_fwd(ptr(enc_pos), B, lay.Te, K, lay.ins, *[ptr(self.p(pm + n)) for n in (
                    "0.weight", "0.bias", "2.weight", "2.bias", "4.weight", "4.bias")], ptr(S["Xv"]), ptr(S["v1"]),
                    ptr(S["v2"]), ptr(vel0), 3, *[_parr([ptr(self.p(nm + suf)) for nm, _, _ in vf])
                                                  for suf in (".l1.weight", ".l1.bias", ".l2.weight", ".l2.bias")],
                    _parr([ptr(src[nm][0]) for nm, _, _ in vf]), _parr([ptr(src[nm][1]) for nm, _, _ in vf]),
                    _parr([ptr(src[nm][2]) for nm, _, _ in vf]), _iarr([P for _, P, _ in vf]), st)
                if self._merge_roll_rec(lay):
                    # the rollout and the reconstruction decode in one launch
                    with self._p("dec_fwd:recon+rollout", 0, self._dec_bytes(F, lay)):
                        L.paig_decoder_fwd_rollout(
                            lay.cell, ptr(enc_pos) + (lay.ins - 1) * D * 4, lay.Te * D, ptr(vel0), ptr(prm[0]),
                            ptr(prm[1]), ptr(prm[2]), ptr(pvs), B, D, lay.R, ptr(enc_pos), 0, 2 * K, 0, ptr(tmpl),
                            ptr(cont), ptr(bgp), ptr(recons), lay.frame, *x_view, ptr(sse_rec), F, K, h, H, st)
                else:
                    L.paig_rollout_fwd(lay.cell, ptr(enc_pos) + (lay.ins - 1) * D * 4, lay.Te * D, ptr(vel0),
                                       ptr(prm[0]), ptr(prm[1]), ptr(prm[2]), ptr(pvs), B, D, lay.R, st)
                    dec_rec(st)
            else:
                velocity(st)
                vfn_src(st)
                dec_rec(st)
        else:
            sst = self._fork(dev)
            velocity(sst)                  # (side) velocity encoder + rollout
            vfn_src(st)                    # (main) VFN sources, reconstruction decode
            dec_rec(st)
            self._join(dev)

        # ---- rollout decode (all B*R frames in one launch, SSE vs input[:, ins:])
        out = _empty(B * lay.R * lay.frame, dev)
        sse_roll = _empty(B * lay.R, dev)
        dec_fwd = L.paig_decoder_fwd_t8 if tb else L.paig_decoder_fwd
        with self._p("dec_fwd:rollout", 0, self._dec_bytes(B * lay.R, lay, tb or 4)):
            dec_fwd(ptr(pvs) + 2 * D * 4, (lay.R + 1) * 2 * D, 2 * D, lay.R, ptr(tmpl), ptr(cont), ptr(bgp),
                    ptr(out), lay.frame, *tgt_roll, ptr(sse_roll), B * lay.R, K, h, H, st)
        S["x_view"] = x_view

        res = {
            "output_seq": out.view(B, lay.R, 3, H, H),
            "recons_out": recons.view(B, lay.Te, 3, H, H),
            "enc_pos": enc_pos.view(B, lay.Te, D),
            "pos_vel_seq": pvs.view(B, lay.R + 1, 2 * D),
            "enc_masks": masks.view(F, K + 1, H, H),
            "masked_objs": [objs[k * F * 3 * HW:(k + 1) * F * 3 * HW].view(F, 3, H, H) for k in range(K)],
            "sse_rec": sse_rec,
            "sse_roll": sse_roll,
            "template": tmpl.view(K, 1, h, h),
            "contents": cont.view(K, 3, h, h),
            "background_content": bgp.view(1, 3, H, H),
        }
        if not need_saved:
            self._release(S)
        return res, (S if need_saved else None)

    # (K, H, cell) of paig_decoder_fwd_rollout (the one-CU decoder's shapes)
    # -> threads per block (DecFw<K, H>::NT: one rollout sequence per thread)
    _ROLL_REC = {(2, 32, 0): 256, (2, 32, 1): 256, (3, 36, 2): 384, (2, 64, 0): 1024}

    def _merge_roll_rec(self, lay):
        """The rollout and the reconstruction decode share one launch while
        the decode's blocks leave room for the rollout's in one round of four
        blocks per CU (B=100: 500 + 1 blocks; B >= 512 measured 0.4-0.6%
        slower merged).  PAIG_MERGE_ROLL=0: two launches (the A/B)."""
        nt = self._ROLL_REC.get((lay.K, lay.H, lay.cell))
        if nt is None or os.environ.get("PAIG_MERGE_ROLL", "1") == "0":
            return False
        return min((lay.F + 1) // 2, 1024) + -(-lay.B // nt) <= 1024

    def _release(self, S):
        """Drop a forward's U-Net workspace (activations, gradients, max-|x|
        slots, pool codes) once its backward has been queued, or there is
        none; stream order keeps the allocator's next user behind every kernel
        that reads it.  The saved state then admits no second backward
        (retain_graph=True)."""
        S.pop("unet_ws", None)
        S["consumed"] = True

    # probe kinds of paig_unet_*_ex (include/paig_hip.h PAIG_PROBE_*) -> tag prefix
    _PROBE_TAG = {0: "conv_fwd", 1: "conv_bwd", 2: "conv_wgrad", 3: "conv_dgrad"}
    _PROBE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int)

    def _unet_probe(self, S):
        """The per-launch probe callback of the C U-Net interpreter: HIP
        events around every conv launch (KernelProbe) with its algorithmic
        FLOPs and HBM bytes (bench.py's roofline); None when not probing."""
        if self.probe is None:
            return None
        lay, F = S["lay"], S["lay"].F
        open_ = {}

        def cb(ctx, ev, op, conv, kind, cin, cout, Hl, fl):
            if ev == 1:
                open_.pop(op).__exit__(None, None, None)
                return
            ks = self.p(lay.prefix + f"c{conv + 1}.weight").shape[-1]
            flops = 2 * F * cin * cout * ks * ks * Hl * Hl
            up = bool(fl & 32)
            hin = Hl // 2 if up else Hl
            if kind == 0 or kind == 2:     # forward / weight gradient: X and Y (dY) once
                nbytes = 4 * F * (cin * hin * hin + cout * Hl * Hl)
            elif kind == 1:                # fused layer backward: data + weight gradients
                flops *= 2
                if up:   # the half-resolution source (and its ReLU' mask) and dY read, its gradient written
                    nbytes = 4 * F * (cin * hin * hin * (2 if fl & 2 else 1) + cout * Hl * Hl)
                else:    # X and dY read, dX written (+ read when accumulating)
                    nbytes = 4 * F * Hl * Hl * (cin + cout + cin * (2 if fl & 4 else 1))
                    if fl & 64:   # the folded max pool: pooled gradient + window codes
                        nbytes += F * (4 * cout + cout) * (Hl // 2) ** 2
            elif fl & 512:                 # data gradient into the upsample source: dY read, its gradient (+ mask)
                nbytes = 4 * F * (cout * Hl * Hl + cin * (Hl // 2) ** 2 * (2 if fl & 2 else 1))
            else:                          # data gradient: dY read, dX written (+ mask, + accumulate)
                nbytes = 4 * F * Hl * Hl * (cout + cin * (1 + (1 if fl & 2 else 0) + (1 if fl & 4 else 0)))
            c = self._p(f"{self._PROBE_TAG[kind]}:c{conv + 1}", flops, nbytes)
            c.__enter__()
            open_[op] = c

        f = self._PROBE_FN(cb)
        S["_probe_cb"] = f   # alive as long as the saved state
        return ctypes.cast(f, ctypes.c_void_p)

    def _unet_forward(self, S, lay, x_view, st, fuse_head=False):
        """The U-Net over F frames addressed by x_view (frame view pointer,
        stride, group, group stride): the C interpreter of csrc/unet.hip
        (paig_unet_fwd_ex) in one workspace that the backward reuses; S["acts"]
        holds the logits ("LG"), or, fuse_head, the 1x1 head's input ("head":
        c12's / c17's output, which the encoder's fused mask softmax reads)."""
        L = self.L
        F, H, K = lay.F, lay.H, lay.K
        dev = S["dev"]
        cm = S["cm"]
        flags = ((1 if fuse_head else 0) | (0 if S.get("need_saved", True) else 4) |
                 (2 if os.environ.get("PAIG_FUSED_BWD", "1") == "0" else 0) |
                 (16 if os.environ.get("PAIG_UPT", "1") == "0" else 0) |   # A/B: standalone upsample backward
                 (32 if os.environ.get("PAIG_POOL_FOLD", "1") == "0" else 0))   # A/B: standalone pool backward
        Ws = [self.p(lay.prefix + f"c{c + 1}.weight") for c in range(lay.nconv)]
        Bs = [self.p(lay.prefix + f"c{c + 1}.bias") for c in range(lay.nconv)]
        # split path: every conv's forward and dgrad weight images (and the
        # localiser's W2^T for the fused dense tail) in one launch per step
        # (paig_conv_wprep); the interpreter takes them per conv
        wp = {}
        wpf = wpd = None
        if cm == self.CONV_MATH["split"]:
            flags |= 8
            jobs = []
            for c, W_ in enumerate(Ws):
                cout, cin, ks = W_.shape[0], W_.shape[1], W_.shape[-1]
                jobs.append((c, 0, W_, cin, cout, ks))
                if c > 0:   # the dgrad kernel's images (Q10: none for the input layer)
                    jobs.append((c, 1, W_, cout, cin, ks))
            sizes = [int(L.paig_conv_wprep_size(j[3], j[4], j[5])) for j in jobs]
            if self.dense_tail():
                jobs.append((-1, 2, self.p("encoder.l2.weight"), 200, 200, 1))
                sizes.append(2 * 200 * 200)
            buf = torch.empty(sum(-(-n // 8) * 8 for n in sizes), dtype=torch.int16, device=dev)
            outs, off = [], 0
            for j, n in zip(jobs, sizes):
                wp[(j[0], j[1])] = buf.data_ptr() + 2 * off
                outs.append(wp[(j[0], j[1])])
                off += -(-n // 8) * 8   # 16-byte aligned images
            n = len(jobs)
            # deferred: the U-Net's first conv carries the prep in its own
            # launch (PAIG_WPREP_MERGE=0: a separate launch, the A/B)
            wprep = L.paig_conv_wprep_defer if os.environ.get("PAIG_WPREP_MERGE", "1") != "0" else L.paig_conv_wprep
            wprep(n, (ctypes.c_void_p * n)(*[ptr(j[2]) for j in jobs]),
                  (ctypes.c_int * n)(*[j[3] for j in jobs]), (ctypes.c_int * n)(*[j[4] for j in jobs]),
                  (ctypes.c_int * n)(*[j[5] for j in jobs]), (ctypes.c_int * n)(*[j[1] for j in jobs]),
                  (ctypes.c_void_p * n)(*outs), st)
            S["wprep_buf"] = buf
            wpf = _parr([wp[(c, 0)] for c in range(lay.nconv)])
            wpd = _parr([wp.get((c, 1), 0) for c in range(lay.nconv)])
        S["wprep"] = wp
        nb = int(L.paig_unet_workspace_ex(lay.net, F, H, K, cm, flags))
        if nb <= 0:
            raise PaigError(f"paig_unet_workspace_ex: no U-Net for net={lay.net} F={F} H={H} K={K} math={cm}")
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        logits = None if fuse_head else _empty(F * K * lay.HW, dev)
        probe = self._unet_probe(S)
        L.paig_unet_fwd_ex(lay.net, F, H, K, cm, flags, *x_view, _parr([ptr(t) for t in Ws]),
                           _parr([ptr(t) for t in Bs]), ptr(logits), wpf, wpd, ptr(ws), nb, probe, None, st)
        acts = {}
        if fuse_head:
            off = int(L.paig_unet_buffer(lay.net, F, H, K, cm, flags, 0, lay.head_buf))
            acts["head"] = ws[off:off + F * lay.head_ci * lay.HW * 4].view(torch.float32)
        else:
            acts["LG"] = logits
        S.update(acts=acts, head_fused=fuse_head, unet_ws=ws, unet_flags=flags, unet_wp=(wpf, wpd))

    def _unet_grad(self, S, buf, n):
        """The U-Net workspace's gradient buffer `buf` (n floats)."""
        lay = S["lay"]
        off = int(self.L.paig_unet_buffer(lay.net, lay.F, lay.H, lay.K, S["cm"], S["unet_flags"], 1, buf))
        assert off >= 0, f"no gradient buffer {buf} in the U-Net workspace"
        return S["unet_ws"][off:off + n * 4].view(torch.float32)

    def _encoder_forward(self, S, lay, x_view, ws, st):
        """ConvolutionalEncoder.forward (nn/network/blocks.py:77-103) over the
        frames of x_view: U-Net, mask softmax x image, l1/l2, position head."""
        L = self.L
        F, H, HW, K = lay.F, lay.H, lay.HW, lay.K
        dev = S["dev"]
        S["x_view"] = x_view
        self._unet_forward(S, lay, x_view, st, fuse_head=lay.fuse_head)
        acts = S["acts"]
        # ---- mask softmax + masked objects + localiser MLP + position head
        masks = _empty(F * (K + 1) * HW, dev)
        objs = _empty(K * F * 3 * HW, dev)
        pobjs = _empty(K * F * lay.l1_in, dev) if lay.unet else None
        if lay.fuse_head:   # the head conv + cat(ones) + softmax + mask x image (+ AvgPool2d), one launch
            hn = lay.prefix + lay.head_name
            L.paig_head_mask_fwd_ex(ptr(acts["head"]), ptr(self.p(hn + ".weight")), ptr(self.p(hn + ".bias")),
                                    *x_view, ptr(masks), ptr(objs), ptr(pobjs), F, K, lay.head_ci, H, H,
                                    lay.head_flags, st)
        else:
            L.paig_mask_softmax_fwd(ptr(acts["LG"]), *x_view, ptr(masks), ptr(objs), ptr(pobjs), F, K, 3, H, H, st)
        l1_x = pobjs if lay.unet else objs
        h1 = _empty(K * F * 200, dev)
        h2 = _empty(K * F * 200, dev)
        h3 = _empty(K * F * 2, dev)
        if not self.dense_tail():
            self.linear(l1_x, K * F, "encoder.l1", h1, 1, st, ws)
            self.linear(h1, K * F, "encoder.l2", h2, 1, st, ws)
            enc_pos = _empty(F * 2 * K, dev)
            L.paig_head_fwd(ptr(h2), ptr(self.p("encoder.l3.weight")), ptr(self.p("encoder.l3.bias")), ptr(h3),
                            ptr(enc_pos), F, K, 200, float(H / 2), st)
        else:
            # l1 (blocks.py:98) as split-K slabs, then ONE launch for its
            # epilogue, l2 and the position head (blocks.py:99-102)
            S["dense_tail"] = True
            n1, KF = lay.l1_in, K * F
            enc_pos = _empty(F * 2 * K, dev)
            with self._p("gemm_fwd:encoder.l1", 2 * KF * 200 * n1, 4 * (KF * n1 + 200 * n1)):
                nS = L.paig_gemm_parts(0, 1, KF, 200, n1, ptr(l1_x), n1, ptr(self.p("encoder.l1.weight")), n1, ptr(ws),
                                       ws.numel(), self.gemm_math(self.FWD), st)
            if nS <= 0:
                raise PaigError(f"paig_gemm_parts failed (rc={nS}): {L.paig_last_error().decode(errors='replace')}")
            with self._p("dense_tail_fwd", 2 * KF * 200 * 200 + 4 * KF * 200,
                         4 * (nS * KF * 200 + 2 * KF * 200 + 200 * 200 + 2 * KF + 2 * KF)):
                w2t = S.get("wprep", {}).get((-1, 2))   # W2^T from the step's weight-prep launch
                w2 = None if w2t is not None else self.p("encoder.l2.weight")
                if w2t is None:
                    S["w2t"] = _empty(200 * 200, dev)
                    w2t = ptr(S["w2t"])
                L.paig_dense_tail_fwd(ptr(ws), nS, ptr(self.p("encoder.l1.bias")), ptr(h1), ptr(w2), w2t,
                                      ptr(self.p("encoder.l2.bias")), ptr(h2),
                                      ptr(self.p("encoder.l3.weight")), ptr(self.p("encoder.l3.bias")), ptr(h3),
                                      ptr(enc_pos), F, K, 200, float(H / 2), st)
        S.update(masks=masks, objs=objs, l1_x=l1_x, h1=h1, h2=h2, h3=h3, enc_pos=enc_pos)

    # -- a second stream for the per-sequence chains (PAIG_SCHED=0 only) ----
    def _fork(self, dev):
        """Side stream ordered after everything issued so far on the current
        stream; graph capture records the fork as a branch."""
        if self._side is None or self._side.device != dev:
            self._side = torch.cuda.Stream(dev)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        self._side.wait_event(ev)
        return self._side.cuda_stream

    def _one_stream(self):
        """The per-sequence chains (velocity encoder, rollout and their
        backward) and the decoder / VFN work run on ONE stream: inside a
        replayed HIP graph every cross-stream edge costs 5-10 us of idle
        queue even when it is long satisfied (tools/timeline.py), more than
        the concurrent kernels overlapped (they slow each other down), so the
        serial order measured 0.6% faster than the round-2 two-stream order
        (PAIG_SCHED=0).  Probed runs keep one stream too."""
        return os.environ.get("PAIG_SCHED", "2") != "0"

    def _join(self, dev):
        ev = torch.cuda.Event()
        ev.record(self._side)
        torch.cuda.current_stream(dev).wait_event(ev)

    def cell_params(self, lay):
        m = self.model
        dt = m.rollout_cell.dt
        if lay.cell == 0:
            return dt, m.rollout_cell.k, m.rollout_cell.equil
        if lay.cell == 2:
            return dt, m.rollout_cell.g, m.rollout_cell.m
        return dt, None, None

    # -- backward --------------------------------------------------------
    def backward(self, S, d_sse_rec=None, d_sse_roll=None, d_out=None, d_recons=None, d_enc_pos=None, d_pvs=None,
                 roll_live=0, lossw=None):
        """Writes every live parameter gradient into the model's flat grad buffer.
        roll_live > 0: only the first roll_live rollout steps of every
        sequence have a loss weight (the others' d_sse_roll entries are zero
        and there is no dense d_out): the rollout decoder backward reads only
        those frames.  lossw: {"rec" / "roll": (mode, (dt, de, dr, ae, B, Te,
        R, pred))} -- that decoder forms its per-frame weights in-kernel from
        the loss adjoints (paig_decoder_bwd_ex) instead of reading d_sse_*."""
        self._check_fresh(S)
        lay = S["lay"]
        L = self.L
        x = S["x"]
        dev = x.device
        st = stream_handle(dev)
        ws = S["ws"]
        S["extra_slabs"] = []   # partial-gradient slabs reduced with the U-Net's at the end
        K, F, HW, H, h, D, B, R = lay.K, lay.F, lay.HW, lay.H, lay.h, lay.D, lay.B, lay.R
        tmpl = S["src"]["var_net_template"][1]
        cont = S["src"]["var_net_content"][1]
        bgp = S["src"]["var_net_background"][2]
        tb = S["tb"]
        lossw = lossw or {}

        if lossw and (K, H) not in ((2, 32), (3, 36), (2, 64)):
            # in-kernel weights need the one-CU decoders: materialise them here
            for key in list(lossw):
                mode, (dt, de, dr, ae, lB, lTe, lR, lpred) = lossw.pop(key)
                w = _empty(lB * (lTe if mode == 1 else lR), dev)
                L.paig_loss_bwd(ptr(dt), ptr(de), ptr(dr), float(ae), ptr(w) if mode == 1 else None,
                                ptr(w) if mode == 2 else None, lB, lTe, lR, lpred, st)
                if mode == 1:
                    d_sse_rec = w
                else:
                    d_sse_roll = w

        def dec_bwd(q, pos, po, pi, pg, tgt, dsse, lw, dout, dpos, slab_p, scr, nfr, live):
            """paig_decoder_bwd_ex: fp32 (4-tuple) or byte (5-tuple) targets; lw:
            in-kernel loss weights or None (dsse read)"""
            tf, t8, ti = (tgt[0], None, None) if len(tgt) == 4 else (None, tgt[0], tgt[1])
            fs, grp, gs = tgt[-3:]
            if lw is not None:
                mode, (dt, de, dr, ae, lB, lTe, lR, lpred) = lw
                lwa = (mode, ptr(dt), ptr(de), ptr(dr), float(ae), lB, lTe, lR, lpred)
                dsse = None
            else:
                lwa = (0, None, None, None, 0.0, 0, 0, 0, 0)
            L.paig_decoder_bwd_ex(pos, po, pi, pg, ptr(tmpl), ptr(cont), ptr(bgp), tf, t8, ti, fs, grp, gs, ptr(dsse),
                                  *lwa, ptr(dout), lay.frame, dpos, slab_p, scr, nfr, live, K, h, H, q)
        if d_out is not None:
            d_out = d_out.contiguous()
        if d_recons is not None:
            d_recons = d_recons.contiguous()

        # ---- buffers of the whole decoder / rollout / velocity backward (all
        # allocated on the main stream before the fork below)
        slab_len = int(L.paig_decoder_slab_len(K, h, H))
        roll_live = roll_live if (d_out is None and 0 < roll_live < R) else 0
        S["roll_live"] = roll_live
        nb_rec = L.paig_decoder_bwd_blocks(F, 0, 0, K, h, H)
        nb_roll = L.paig_decoder_bwd_blocks(B * R, R, roll_live, K, h, H)
        slab = _empty((nb_rec + nb_roll) * slab_len, dev)
        scr_n = max(L.paig_decoder_bwd_scratch(F, K, h, H), L.paig_decoder_bwd_scratch(B * R, K, h, H))
        scratch = _empty(scr_n, dev) if scr_n else None
        denc = _empty(F * D, dev)   # d enc_pos [B][Te][D]
        dpos_roll = _empty(B * R * D, dev)
        dsrc = _empty(slab_len, dev)
        pvs = S["pvs"]
        dpos0 = _empty(B * D, dev)
        dvel0 = _empty(K * B * 2, dev) if S["vel0"] is not None else None
        rpart = _empty(2 * L.paig_rollout_bwd_blocks(B), dev, torch.float64)
        dXv = vslab = None
        if S["vel0"] is not None:
            dXv = _empty(K * B * 2 * (lay.ins - 1 if lay.alt_vel else lay.ins), dev)
            if not lay.alt_vel:
                vblk, vlen = L.paig_velmlp_bwd_blocks(K * B), L.paig_velmlp_slab_len(lay.ins)
                vslab = _empty(vblk * vlen, dev)
        vfn = (("var_net_template", K * h * h, 0, tmpl), ("var_net_content", K * 3 * h * h, 1, cont),
               ("var_net_background", 3 * HW, 1, S["src"]["var_net_background"][1]))
        vparts = [_empty(L.paig_vfn_bwd_blocks(P) * 200, dev) for _, P, _, _ in vfn]

        prm = self.cell_params(lay)
        gk = gq = None
        if lay.cell == 0:
            gk, gq = self.g("rollout_cell.k"), self.g("rollout_cell.equil")
        elif lay.cell == 2:
            gk = self.g("rollout_cell.g")
        # the chains' inputs exist before any fork (a temporary made after it
        # could be recycled by a main-stream allocation while a side kernel
        # still reads it)
        d_pvs_c = d_pvs.contiguous() if d_pvs is not None else None
        d_enc_c = d_enc_pos.contiguous() if d_enc_pos is not None else None
        live_frames = B * roll_live if roll_live else B * R

        def dec_roll(q):   # rollout-frame decoder backward: d rollout positions + partial source grads
            with self._p("dec_bwd:rollout", 0, self._dec_bwd_bytes(live_frames, B * R, lay, d_out is not None, tb or 4)):
                dec_bwd(q, ptr(pvs) + 2 * D * 4, (R + 1) * 2 * D, 2 * D, R, S["tgt_roll"], d_sse_roll,
                        lossw.get("roll"), d_out, ptr(dpos_roll), ptr(slab) + nb_rec * slab_len * 4, ptr(scratch),
                        B * R, roll_live)

        def dec_rec(q):    # reconstruction decoder backward: d enc_pos + partial source grads
            with self._p("dec_bwd:recon", 0, self._dec_bwd_bytes(F, F, lay, d_recons is not None)):
                dec_bwd(q, ptr(S["enc_pos"]), 0, 2 * K, 0, S["x_view"], d_sse_rec, lossw.get("rec"), d_recons,
                        ptr(denc), ptr(slab), ptr(scratch), F, 0)

        def physics(q):    # rollout adjoint -> d pos0, d vel0, physics params; velocity encoder backward
            L.paig_rollout_bwd(lay.cell, ptr(pvs), ptr(dpos_roll), ptr(d_pvs_c), ptr(prm[0]), ptr(prm[1]),
                               ptr(prm[2]), ptr(dpos0), ptr(dvel0), ptr(rpart), ptr(gk), ptr(gq), 0, B, D, R, q)
            if S["vel0"] is not None:
                if lay.alt_vel:
                    self.linear_bwd(S["Xv"], dvel0, K * B, "velocity_encoder.init_vel_linear", dXv, None, 0, q, ws)
                else:   # one launch; its partial weight grads join the U-Net's batched slab reduction
                    pm = "velocity_encoder.init_vel_mlp."
                    L.paig_velmlp_bwd(ptr(dvel0), ptr(S["Xv"]), ptr(S["v1"]), ptr(S["v2"]),
                                      ptr(self.p(pm + "0.weight")), ptr(self.p(pm + "2.weight")),
                                      ptr(self.p(pm + "4.weight")), ptr(dXv), ptr(vslab), K * B, lay.ins, q)
                    g0 = self.g(pm + "0.weight")
                    assert self.g(pm + "4.bias").data_ptr() == g0.data_ptr() + (vlen - 2) * 4, \
                        "velocity MLP grads not contiguous"
                    S["extra_slabs"].append((vslab, vblk, vlen, g0))

        def sources(q, split=False):   # source-gradient reduction (both decoders' slab rows), VFN backward
            L.paig_slab_reduce_multi(1, (ctypes.c_void_p * 1)(ptr(slab)), (ctypes.c_int * 1)(nb_rec + nb_roll),
                                     (ctypes.c_int * 1)(slab_len), (ctypes.c_void_p * 1)(ptr(dsrc)), 0, q)
            offs = [0, vfn[0][1], vfn[0][1] + vfn[1][1]]
            args = (3, _parr([ptr(dsrc) + o * 4 for o in offs]), _parr([ptr(r) for _, _, _, r in vfn]),
                    _iarr([sg for _, _, sg, _ in vfn]),
                    _parr([ptr(S["src"][nm][0]) for nm, _, _, _ in vfn]),
                    _parr([ptr(self.p(nm + ".l2.weight")) for nm, _, _, _ in vfn]),
                    *[_parr([ptr(self.g(nm + suf)) for nm, _, _, _ in vfn])
                      for suf in (".l1.weight", ".l1.bias", ".l2.weight", ".l2.bias")],
                    _parr([ptr(pt) for pt in vparts]), _iarr([P for _, P, _, _ in vfn]))
            if split:      # phase 1 here, phase 2 inside the head backward's launch
                L.paig_vfn_bwd1_multi(*args, q)
                return args
            L.paig_vfn_bwd_multi(*args, q)
            return None

        if self._one_stream():
            dec_roll(st)
            physics(st)
            dec_rec(st)
            fuse_vel = os.environ.get("PAIG_FUSE_VEL", "1") != "0"
            # VFN backward phase 2 inside the head backward's launch
            vfn2 = sources(st, split=fuse_vel and os.environ.get("PAIG_FUSE_VFN2", "1") != "0")
            if d_enc_c is not None:
                L.paig_axpby(ptr(d_enc_c), ptr(denc), F * D, 1.0, 1.0, st)
            # the velocity encoder's input gradient is added inside the head
            # backward (PAIG_FUSE_VEL=0: the separate unpack-add launch)
            vel = (dXv, dpos0, B, lay.Te, lay.ins, int(lay.alt_vel), vfn2)
            if not fuse_vel:
                L.paig_vel_unpack_add(ptr(dXv), ptr(dpos0), ptr(denc), B, lay.Te, K, lay.ins, int(lay.alt_vel), st)
                vel = None
        else:
            dec_roll(st)
            sst = self._fork(dev)
            physics(sst)   # (side) rollout adjoint + velocity encoder backward
            dec_rec(st)    # (main) reconstruction decoder backward, source reduction, VFN backward
            sources(st)
            if d_enc_c is not None:
                L.paig_axpby(ptr(d_enc_c), ptr(denc), F * D, 1.0, 1.0, st)
            self._join(dev)
            L.paig_vel_unpack_add(ptr(dXv), ptr(dpos0), ptr(denc), B, lay.Te, K, lay.ins, int(lay.alt_vel), st)
            vel = None
        del d_pvs_c, d_enc_c   # (kept alive across the side chain)

        self._encoder_backward(S, denc, st, vel=vel)

    def _encoder_backward(self, S, denc, st, hook=True, vel=None):
        """ConvolutionalEncoder backward from d enc_pos (denc [F][2K]): position
        head, l2/l1, mask softmax, U-Net; all its weight gradients."""
        lay = S["lay"]
        L = self.L
        dev = S["dev"]
        ws = S["ws"]
        K, F, HW, H = lay.K, lay.F, lay.HW, lay.H
        x_view = S["x_view"]
        S.setdefault("extra_slabs", [])
        # ---- position head + localiser MLP backward -> d masked objects
        dh2 = _empty(K * F * 200, dev)
        dh1 = _empty(K * F * 200, dev)
        fused_l2 = S.get("dense_tail", False)   # l2's data gradient formed inside the head backward's launch
        hblk = L.paig_head_l2_bwd_blocks(K * F) if fused_l2 else L.paig_head_bwd_blocks(K * F)
        hslab = _empty(hblk * (2 * 200 + 2), dev)
        if fused_l2:
            dXv = dpos0 = None
            Bv = Tev = Sv = altv = 0
            vfn2 = None
            if vel is not None:
                dXv, dpos0, Bv, Tev, Sv, altv, vfn2 = vel
            vf = vfn2 if vfn2 is not None else (0,) + (None,) * 11
            L.paig_head_l2_bwd(ptr(S["h2"]), ptr(S["h3"]), ptr(denc), ptr(self.p("encoder.l3.weight")), ptr(dh2),
                               ptr(hslab), F, K, 200, float(H / 2), ptr(dXv) if torch.is_tensor(dXv) else dXv,
                               ptr(dpos0) if torch.is_tensor(dpos0) else dpos0, Bv, Tev, Sv, altv,
                               ptr(self.p("encoder.l2.weight")), ptr(S["h1"]), ptr(dh1), *vf, st)
        elif vel is not None and vel[6] is not None:   # + the VFN backward's phase 2
            dXv, dpos0, Bv, Tev, Sv, altv, vfn2 = vel
            L.paig_head_bwd_vel_vfn2(ptr(S["h2"]), ptr(S["h3"]), ptr(denc), ptr(self.p("encoder.l3.weight")),
                                     ptr(dh2), ptr(hslab), F, K, 200, float(H / 2), ptr(dXv), ptr(dpos0), Bv, Tev,
                                     Sv, altv, *vfn2, st)
        elif vel is not None:   # + the velocity encoder's input gradient (dXv, dpos0, B, Te, S, alt)
            dXv, dpos0, Bv, Tev, Sv, altv, _ = vel
            L.paig_head_bwd_vel(ptr(S["h2"]), ptr(S["h3"]), ptr(denc), ptr(self.p("encoder.l3.weight")), ptr(dh2),
                                ptr(hslab), F, K, 200, float(H / 2), ptr(dXv), ptr(dpos0), Bv, Tev, Sv, altv, st)
        else:
            L.paig_head_bwd(ptr(S["h2"]), ptr(S["h3"]), ptr(denc), ptr(self.p("encoder.l3.weight")), ptr(dh2),
                            ptr(hslab), F, K, 200, float(H / 2), st)
        g3 = self.g("encoder.l3.weight")
        assert self.g("encoder.l3.bias").data_ptr() == g3.data_ptr() + 400 * 4, "l3 grads not contiguous"
        S["extra_slabs"].append((hslab, hblk, 402, g3))
        dobjs = _empty(K * F * lay.l1_in, dev)
        # l2's weight-gradient epilogue rides in l1's weight-gradient launch, and
        # l1's in l1's data-gradient launch (neither reads the deferred output;
        # l1's weight gradient takes the workspace past l2's partial slabs).
        # PAIG_GEMM_EPI_MERGE=0: separate epilogue launches (the A/B)
        merge = os.environ.get("PAIG_GEMM_EPI_MERGE", "1") != "0" and not self.probe
        w2 = int(L.paig_gemm_workspace(200, 200, K * F)) if merge else 0
        self.linear_bwd(S["h1"], dh2, K * F, "encoder.l2", dh1, S["h1"], 1, st, ws, need_dx=not fused_l2,
                        defer_epi=merge)
        self.linear_bwd(S["l1_x"], dh1, K * F, "encoder.l1", dobjs, None, 0, st, ws[w2:] if merge else ws,
                        defer_epi=merge)
        if merge:
            L.paig_gemm_flush(st)
        # every gradient of the flat buffer's early bucket is final (queued on
        # this stream): the data-parallel all-reduce of that bucket may start
        if hook and self.bucket_hook is not None:
            self.bucket_hook()

        # ---- mask softmax backward (incl. ReLU' of ShallowUNet's c13, Q13, and
        # the AvgPool2d backward of the UNet path)
        acts = S["acts"]
        if S.get("head_fused"):
            # fused head + softmax backward: the head input's dY (its
            # producer's ReLU' applied), written straight into the U-Net
            # workspace's gradient buffer, and the head's weight/bias partials
            # (one slab row per block)
            hn, c = lay.prefix + lay.head_name, lay.head_ci
            dXl = self._unet_grad(S, lay.head_buf, F * c * HW)
            nb = L.paig_head_mask_blocks(F, H, H)
            nw = K * c + K
            hs = _empty(nb * nw, dev)
            L.paig_head_mask_bwd_ex(ptr(acts["head"]), ptr(self.p(hn + ".weight")), ptr(self.p(hn + ".bias")),
                                    *x_view, ptr(S["masks"]), ptr(dobjs), ptr(dXl), ptr(hs), F, K, c, H, H,
                                    lay.head_flags, st)
            gh = self.g(hn + ".weight")
            assert self.g(hn + ".bias").data_ptr() == gh.data_ptr() + K * c * 4, "head grads not contiguous"
            S["extra_slabs"].append((hs, nb, nw, gh))
            self._unet_backward(S, None, st)
        else:
            dLG = _empty(F * K * HW, dev)
            L.paig_mask_softmax_bwd(ptr(acts["LG"]), x_view[0], x_view[1], x_view[2], x_view[3], ptr(S["masks"]),
                                    ptr(dobjs), ptr(dLG), F, K, 3, H, H,
                                    (1 if lay.lg_relu else 0) | (2 if lay.unet else 0), st)
            self._unet_backward(S, dLG, st)

    @staticmethod
    def _check_fresh(S):
        if S.get("consumed"):
            raise PaigError("a second backward through one forward (retain_graph=True) is not supported: the "
                            "forward's saved state (its U-Net workspace) was released by the first backward")

    def _unet_backward(self, S, dlogits, st):
        """The U-Net backward (paig_unet_bwd_ex, the same C interpreter as the
        forward) from d logits, or (fused head) from the head input's
        gradient already in the workspace; every conv's weight and bias
        gradient, with the step's other partial-gradient slabs (extra_slabs:
        head, l3, velocity MLP) in one batched deterministic reduction."""
        self._check_fresh(S)
        lay = S["lay"]
        L = self.L
        Ws = [self.p(lay.prefix + f"c{c + 1}.weight") for c in range(lay.nconv)]
        dwb = []
        for c in range(lay.nconv):
            gw = self.g(lay.prefix + f"c{c + 1}.weight")
            assert self.g(lay.prefix + f"c{c + 1}.bias").data_ptr() == gw.data_ptr() + gw.numel() * 4, \
                "flat grads: weight and bias must be adjacent"
            dwb.append(ptr(gw))
        extra = S.get("extra_slabs", [])
        n = len(extra)
        ws = S["unet_ws"]
        _, wpd = S["unet_wp"]
        L.paig_unet_bwd_ex(lay.net, lay.F, lay.H, lay.K, S["cm"], S["unet_flags"], *S["x_view"],
                           _parr([ptr(t) for t in Ws]), ptr(S["acts"].get("LG")), ptr(dlogits), _parr(dwb), n,
                           _parr([ptr(e[0]) for e in extra]), _iarr([e[1] for e in extra]),
                           _iarr([e[2] for e in extra]), _parr([ptr(e[3]) for e in extra]), wpd, ptr(ws), ws.numel(),
                           self._unet_probe(S), None, st)
        self._release(S)
