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

from ._lib import XMAX_SLOTS, PaigError, lib, ptr, stream_handle, require_device

# --------------------------------------------------------------------------
# U-Net plans (buffers + ops), forward order.  A buffer is (channels, level),
# level = spatial divisor.  An op's src/dst are (buffer, channel offset, count).
# --------------------------------------------------------------------------


def _conv(name, src, dst, relu, ks=3):
    return {"op": "conv", "name": name, "src": src, "dst": dst, "relu": relu, "ks": ks}


def _pool(src, dst):
    return {"op": "pool", "src": src, "dst": dst}


def _up(src, dst):
    return {"op": "up", "src": src, "dst": dst}


def shallow_unet_plan(c, K):
    """ShallowUNet, nn/network/blocks.py:240-308 (hidden c=8; c13 ReLU'd, Q13)."""
    bufs = {"X0": (3, 1), "A1": (c, 1), "CAT2": (3 * c, 1), "P1": (c, 2), "A3": (2 * c, 2), "CAT1": (4 * c, 2),
            "P2": (2 * c, 4), "A5": (4 * c, 4), "A6": (4 * c, 4), "U1": (4 * c, 2), "A8": (2 * c, 2),
            "A9": (2 * c, 2), "U2": (2 * c, 1), "A11": (c, 1), "A12": (c, 1), "LG": (K, 1)}
    ops = [
        _conv("c1", ("X0", 0, 3), ("A1", 0, c), True),
        _conv("c2", ("A1", 0, c), ("CAT2", 2 * c, c), True),
        _pool(("CAT2", 2 * c, c), ("P1", 0, c)),
        _conv("c3", ("P1", 0, c), ("A3", 0, 2 * c), True),
        _conv("c4", ("A3", 0, 2 * c), ("CAT1", 2 * c, 2 * c), True),
        _pool(("CAT1", 2 * c, 2 * c), ("P2", 0, 2 * c)),
        _conv("c5", ("P2", 0, 2 * c), ("A5", 0, 4 * c), True),
        _conv("c6", ("A5", 0, 4 * c), ("A6", 0, 4 * c), True),
        _up(("A6", 0, 4 * c), ("U1", 0, 4 * c)),
        _conv("c7", ("U1", 0, 4 * c), ("CAT1", 0, 2 * c), False),
        _conv("c8", ("CAT1", 0, 4 * c), ("A8", 0, 2 * c), True),
        _conv("c9", ("A8", 0, 2 * c), ("A9", 0, 2 * c), True),
        _up(("A9", 0, 2 * c), ("U2", 0, 2 * c)),
        _conv("c10", ("U2", 0, 2 * c), ("CAT2", 0, 2 * c), False),
        _conv("c11", ("CAT2", 0, 3 * c), ("A11", 0, c), True),
        _conv("c12", ("A11", 0, c), ("A12", 0, c), True),
        _conv("c13", ("A12", 0, c), ("LG", 0, K), True, ks=1),
    ]
    return bufs, ops


def unet_plan(h, K):
    """UNet, nn/network/blocks.py:106-237 (hidden h=16; c9/c12/c15/c18 un-ReLU'd)."""
    bufs = {"X0": (3, 1), "A1": (h, 1), "CAT3": (3 * h, 1), "P1": (h, 2), "A3": (2 * h, 2), "CAT2": (4 * h, 2),
            "P2": (2 * h, 4), "A5": (4 * h, 4), "CAT1": (6 * h, 4), "P3": (4 * h, 8), "A7": (8 * h, 8),
            "A8": (8 * h, 8), "U1": (8 * h, 4), "A10": (4 * h, 4), "A11": (4 * h, 4), "U2": (4 * h, 2),
            "A13": (2 * h, 2), "A14": (2 * h, 2), "U3": (2 * h, 1), "A16": (h, 1), "A17": (h, 1), "LG": (K, 1)}
    ops = [
        _conv("c1", ("X0", 0, 3), ("A1", 0, h), True),
        _conv("c2", ("A1", 0, h), ("CAT3", 2 * h, h), True),
        _pool(("CAT3", 2 * h, h), ("P1", 0, h)),
        _conv("c3", ("P1", 0, h), ("A3", 0, 2 * h), True),
        _conv("c4", ("A3", 0, 2 * h), ("CAT2", 2 * h, 2 * h), True),
        _pool(("CAT2", 2 * h, 2 * h), ("P2", 0, 2 * h)),
        _conv("c5", ("P2", 0, 2 * h), ("A5", 0, 4 * h), True),
        _conv("c6", ("A5", 0, 4 * h), ("CAT1", 2 * h, 4 * h), True),
        _pool(("CAT1", 2 * h, 4 * h), ("P3", 0, 4 * h)),
        _conv("c7", ("P3", 0, 4 * h), ("A7", 0, 8 * h), True),
        _conv("c8", ("A7", 0, 8 * h), ("A8", 0, 8 * h), True),
        _up(("A8", 0, 8 * h), ("U1", 0, 8 * h)),
        _conv("c9", ("U1", 0, 8 * h), ("CAT1", 0, 2 * h), False),
        _conv("c10", ("CAT1", 0, 6 * h), ("A10", 0, 4 * h), True),
        _conv("c11", ("A10", 0, 4 * h), ("A11", 0, 4 * h), True),
        _up(("A11", 0, 4 * h), ("U2", 0, 4 * h)),
        _conv("c12", ("U2", 0, 4 * h), ("CAT2", 0, 2 * h), False),
        _conv("c13", ("CAT2", 0, 4 * h), ("A13", 0, 2 * h), True),
        _conv("c14", ("A13", 0, 2 * h), ("A14", 0, 2 * h), True),
        _up(("A14", 0, 2 * h), ("U3", 0, 2 * h)),
        _conv("c15", ("U3", 0, 2 * h), ("CAT3", 0, 2 * h), False),
        _conv("c16", ("CAT3", 0, 3 * h), ("A16", 0, h), True),
        _conv("c17", ("A16", 0, h), ("A17", 0, h), True),
        _conv("c18", ("A17", 0, h), ("LG", 0, K), False, ks=1),
    ]
    return bufs, ops


def _overlap(a, b):
    return a[0] == b[0] and a[1] < b[1] + b[2] and b[1] < a[1] + a[2]


def backward_plan(ops):
    """For every op, the producer regions of its source that it FINALIZES
    (it is their earliest consumer in forward order = last in reverse), so a
    ReLU derivative is applied exactly once, after all contributions."""
    producers = [(i, op["dst"], op.get("relu", False)) for i, op in enumerate(ops)]
    fin = {i: [] for i in range(len(ops))}
    for pi, region, relu in producers:
        consumers = [i for i, op in enumerate(ops) if i > pi and _overlap(op["src"], region)]
        if consumers:
            fin[min(consumers)].append((region, relu))
    return fin


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
        if self.unet:       # UNet(hidden 16), blocks.py:106-237; c18 not ReLU'd
            self.bufs, self.ops = unet_plan(16, self.K)
            self.prefix = "encoder.unet."
        else:               # ShallowUNet(hidden 8), blocks.py:240-308; c13 ReLU'd (Q13)
            self.bufs, self.ops = shallow_unet_plan(8, self.K)
            self.prefix = "encoder.shallow_unet."
        self.lg_relu = not self.unet
        # l1 input: the masked objects, AvgPool2d(2)'d first for H >= 40 (blocks.py:92-96)
        self.l1_in = 3 * (self.H // 2) ** 2 if self.unet else 3 * self.H * self.H
        self.fin = backward_plan(self.ops)
        # an upsample consumed by exactly one conv is fused into that conv's
        # input staging (fwd and wgrad) when the MFMA path has the shape; only
        # the gradient buffer of the upsampled tensor remains (dgrad output ->
        # upsample backward)
        L = lib()
        self.fused_up, self.fused_bufs = {}, set()
        for i, op in enumerate(self.ops):
            if op["op"] != "up":
                continue
            consumers = [j for j, o in enumerate(self.ops) if o["src"][0] == op["dst"][0]]
            if len(consumers) != 1 or self.ops[consumers[0]]["op"] != "conv":
                continue
            c = self.ops[consumers[0]]
            Hc = self.H // self.bufs[op["dst"][0]][1]
            cm = Engine.CONV_MATH.get(getattr(model, "conv_math", "split"), 0)
            if all(L.paig_conv2d_mfma_supported(w, c["src"][2], c["dst"][2], Hc, Hc, c["ks"], 32 | cm) for w in (0, 1)):
                self.fused_up[consumers[0]] = op
                self.fused_bufs.add(op["dst"][0])
        self.HW = self.H * self.H
        self.frame = 3 * self.HW
        # ShallowUNet: c13 (1x1, 8 -> K) is fused into the mask softmax
        # (paig_head_mask_fwd/bwd) in the encoder; the standalone U-Net call
        # keeps it as a conv (its logits are the output)
        last = self.ops[-1]
        self.fuse_head = (not self.unet and last["name"] == "c13" and last["ks"] == 1 and last["src"][2] == 8
                          and self.K in (2, 3) and self.HW % 4 == 0)


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
        self._xmax = {}     # per-layout xmax slots (see _unet_forward)
        # called once per backward when the early gradient bucket is final
        # (FlatParams.allreduce_early by default; bench.py splits its HIP graph here)
        self.bucket_hook = model._flat.allreduce_early

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
    def _dec_bytes(n, lay):
        """Algorithmic HBM bytes of one decoder forward over n frames: the
        target frames read (fused SSE) and the decoded frames written;
        positions and the step-constant sources (< 100 KB) are negligible."""
        return 2 * n * lay.frame * 4

    @staticmethod
    def _dec_bwd_bytes(live, n, lay, dense):
        """Algorithmic HBM bytes of one decoder backward: the targets of the
        `live` frames that carry a loss weight (+ their dense dL/dout when
        given) read, the position gradients of all n frames and the source
        gradients (one slab_len vector) written.  The partial-gradient slab
        rows are the kernel's own overhead, not algorithmic."""
        return live * lay.frame * 4 * (2 if dense else 1) + n * 2 * lay.D * 4 + (4 * lay.K * lay.h * lay.h + 3 * lay.HW) * 4

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

    def linear_bwd(self, x, dy, rows, name, dx, aux, auxm, st, ws, need_dx=True):
        """dW = dy^T x and db = colsum(dy) (one GEMM, fused row sums) ; dx = (dy W) * act'(aux)"""
        W = self.p(name + ".weight")
        O, I = W.shape
        gW, gb = self.g(name + ".weight"), self.g(name + ".bias")
        n_ws = ws.numel()
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
                                   lay.frame, x_view[0], x_view[1], x_view[2], x_view[3], ptr(sse_rec), F, K, h, H, q)

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
                L.paig_rollout_fwd(lay.cell, ptr(enc_pos) + (lay.ins - 1) * D * 4, lay.Te * D, ptr(vel0),
                                   ptr(prm[0]), ptr(prm[1]), ptr(prm[2]), ptr(pvs), B, D, lay.R, st)
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
        tgt_roll = (ptr(x) + lay.ins * lay.frame * 4, T * lay.frame, lay.R, lay.frame)
        with self._p("dec_fwd:rollout", 0, self._dec_bytes(B * lay.R, lay)):
            L.paig_decoder_fwd(ptr(pvs) + 2 * D * 4, (lay.R + 1) * 2 * D, 2 * D, lay.R, ptr(tmpl), ptr(cont),
                               ptr(bgp), ptr(out), lay.frame, *tgt_roll, ptr(sse_roll), B * lay.R, K, h, H, st)
        S["tgt_roll"] = tgt_roll
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
            self._release_xmax(S)
        return res, (S if need_saved else None)

    def _release_xmax(self, S):
        """Return a forward's xmax slots to the free list (its backward has
        been queued, or there is none); stream order keeps the next user
        behind every kernel that reads them."""
        buf = S.pop("xmax_buf", None)
        if buf is not None:
            self._xmax.setdefault(S["xmax_key"], []).append(buf)
        # the slots may now be another forward's: this forward's saved state
        # admits no second backward (retain_graph=True)
        S["consumed"] = True

    def _unet_forward(self, S, lay, x_view, st, fuse_head=False):
        """The U-Net plan over F frames addressed by x_view (frame view
        pointer, stride, group, group stride): fills S["acts"] (LG = logits).
        fuse_head: stop before the last op (ShallowUNet's c13), which the
        encoder runs fused into the mask softmax (no LG buffer)."""
        L = self.L
        F, H = lay.F, lay.H
        dev = S["dev"]
        cm = S["cm"]
        acts = {}
        S["head_fused"] = fuse_head
        ops = lay.ops[:-1] if fuse_head else lay.ops
        for name, (C, lvl) in lay.bufs.items():
            if fuse_head and name == "LG":
                continue
            if name != "X0" and name not in lay.fused_bufs:
                acts[name] = _empty(F * C * (H // lvl) * (H // lvl), dev)
        S["acts"] = acts

        def view(region):
            buf, off, n = region
            C, lvl = lay.bufs[buf]
            hw = (H // lvl) ** 2
            if buf == "X0":
                return (x_view[0] + off * hw * 4, x_view[1], x_view[2], x_view[3]), lvl
            t = acts[buf]
            return (t.data_ptr() + off * hw * 4, C * hw, 0, 0), lvl

        def conv_input(i, op):
            """(view, level of the conv, extra flags): a fused upsample reads its
            half-resolution source and forms the 2x bilinear rows while staging."""
            up = lay.fused_up.get(i)
            if up is None:
                v, lvl = view(op["src"])
                return v, lvl, 0
            v, lvl = view(up["src"])
            return v, lvl // 2, 32

        S["view"] = view
        S["conv_input"] = conv_input
        # per conv: the split forward's per-block max |input| slots, which
        # set the X scale of the same input's wgrad (every slot is written;
        # zeroed so that a slot no forward wrote falls back to the guarded
        # fixed scale instead of a garbage exponent).  Each forward owns its
        # buffer until its backward has consumed it (a second forward before
        # the first one's backward takes another); buffers return to a
        # per-(device, layout) free list, so steady-state steps reuse one
        # buffer (a step of the same shape rewrites exactly the same slots)
        # and the zero fill (an extra launch) happens once.
        key = (str(dev), len(lay.ops), lay.F, lay.H)
        free = self._xmax.setdefault(key, [])
        xmax = free.pop() if free else torch.zeros(len(lay.ops) * XMAX_SLOTS, device=dev)
        S["xmax"] = lambda i: ptr(xmax) + i * XMAX_SLOTS * 4
        S["xmax_buf"] = xmax
        S["xmax_key"] = key
        # split path: every conv's forward and dgrad weight images, pre-split
        # in one launch per step (paig_conv_wprep) and copied by the kernels
        wp = {}
        if cm == self.CONV_MATH["split"]:
            jobs = []
            for i, op in enumerate(ops):
                if op["op"] != "conv":
                    continue
                W_ = self.p(lay.prefix + op["name"] + ".weight")
                cin, cout, ks = op["src"][2], op["dst"][2], op["ks"]
                jobs.append((i, 0, W_, cin, cout, ks))
                if op["src"][0] != "X0":   # the dgrad kernel's images (Q10: none for the input)
                    jobs.append((i, 1, W_, cout, cin, ks))
            sizes = [int(L.paig_conv_wprep_size(j[3], j[4], j[5])) for j in jobs]
            if self.dense_tail():
                # the localiser's W2^T for the fused dense tail, in the same launch
                jobs.append((-1, 2, self.p("encoder.l2.weight"), 200, 200, 1))
                sizes.append(2 * 200 * 200)
            buf = torch.empty(sum(-(-n // 8) * 8 for n in sizes), dtype=torch.int16, device=dev)
            outs, off = [], 0
            for j, n in zip(jobs, sizes):
                wp[(j[0], j[1])] = buf.data_ptr() + 2 * off
                outs.append(wp[(j[0], j[1])])
                off += -(-n // 8) * 8   # 16-byte aligned images
            n = len(jobs)
            L.paig_conv_wprep(n, (ctypes.c_void_p * n)(*[ptr(j[2]) for j in jobs]),
                              (ctypes.c_int * n)(*[j[3] for j in jobs]), (ctypes.c_int * n)(*[j[4] for j in jobs]),
                              (ctypes.c_int * n)(*[j[5] for j in jobs]), (ctypes.c_int * n)(*[j[1] for j in jobs]),
                              (ctypes.c_void_p * n)(*outs), st)
            S["wprep_buf"] = buf
        S["wprep"] = wp
        pooled = set()   # pools written by their producing conv's epilogue
        for i, op in enumerate(ops):
            if op["op"] == "up" and op["dst"][0] in lay.fused_bufs:
                continue   # formed inside the consuming conv's staging
            if i in pooled:
                continue
            dv, dlvl = view(op["dst"])
            if op["op"] == "conv":
                sv, clvl, xfl = conv_input(i, op)
                Hl = H // clvl
                # a 2x2 max pool of exactly this output, next in the plan, is
                # fused into the conv's epilogue where the split kernel has it
                pool_v = (None, 0)
                nxt = ops[i + 1] if i + 1 < len(ops) else None
                pcode = (None, 0)
                pool_next = nxt is not None and nxt["op"] == "pool" and nxt["src"] == op["dst"] and not xfl and cm
                if pool_next and S.get("need_saved", True) and self._fused_bwd(op["src"][2], op["dst"][2], Hl,
                                                                                 op["ks"], cm | 64):
                    # the pool windows' codes (ReLU' bits + argmax): the
                    # backward folds the pool into this layer's dY staging.
                    # Written by this conv's fused pool, or (widths whose rows
                    # are not whole M-tiles: 3bp) by the standalone pool
                    cfs = -(-op["dst"][2] // 8) * 8 * (Hl // 2) ** 2
                    cb = torch.empty(F * cfs, dtype=torch.uint8, device=dev)
                    S.setdefault("pcode", {})[i + 1] = (cb, cfs)
                    pcode = (cb.data_ptr(), cfs)
                if pool_next and L.paig_conv2d_mfma_supported(0, op["src"][2], op["dst"][2], Hl, Hl, op["ks"],
                                                              cm | 64):
                    pv, _ = view(nxt["dst"])
                    pool_v = (pv[0], pv[1])
                    pooled.add(i + 1)
                else:
                    pcode = (None, 0)
                W_ = self.p(lay.prefix + op["name"] + ".weight")
                b_ = self.p(lay.prefix + op["name"] + ".bias")
                fl = 2 * F * op["src"][2] * op["dst"][2] * op["ks"] ** 2 * Hl * Hl
                nbytes = 4 * F * (op["src"][2] * (Hl // (2 if xfl else 1)) ** 2 + op["dst"][2] * Hl * Hl)
                with self._p("conv_fwd:" + op["name"], fl, nbytes):
                    L.paig_conv2d_fwd_pwc(sv[0], sv[1], sv[2], sv[3], dv[0], dv[1], None, 0, ptr(W_), ptr(b_), F,
                                          op["src"][2], op["dst"][2], Hl, Hl, op["ks"],
                                          (1 if op["relu"] else 0) | xfl | cm | (64 if pool_v[0] else 0),
                                          S["xmax"](i), XMAX_SLOTS, pool_v[0], pool_v[1], pcode[0], pcode[1],
                                          wp.get((i, 0)), st)
            elif op["op"] == "pool":
                sv, slvl = view(op["src"])
                Hl = H // slvl
                if i in S.get("pcode", {}):
                    cb, cfs = S["pcode"][i]
                    L.paig_maxpool2_fwd_codes(sv[0], sv[1], dv[0], dv[1], cb.data_ptr(), cfs, F, op["src"][2], Hl, Hl,
                                              st)
                else:
                    L.paig_maxpool2_fwd(sv[0], sv[1], dv[0], dv[1], F, op["src"][2], Hl, Hl, st)
            else:
                sv, slvl = view(op["src"])
                Hs, Ho = H // slvl, H // dlvl
                L.paig_upsample2_fwd(sv[0], sv[1], dv[0], dv[1], F, op["src"][2], Hs, Hs, Ho, Ho, st)

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
        if lay.fuse_head:   # c13 + cat(ones) + softmax + mask x image, one launch
            L.paig_head_mask_fwd(ptr(acts["A12"]), ptr(self.p(lay.prefix + "c13.weight")),
                                 ptr(self.p(lay.prefix + "c13.bias")), *x_view, ptr(masks), ptr(objs), F, K, H, H, st)
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
                 roll_live=0):
        """Writes every live parameter gradient into the model's flat grad buffer.
        roll_live > 0: only the first roll_live rollout steps of every
        sequence have a loss weight (the others' d_sse_roll entries are zero
        and there is no dense d_out): the rollout decoder backward reads only
        those frames."""
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
        x_view = S["x_view"]
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
            with self._p("dec_bwd:rollout", 0, self._dec_bwd_bytes(live_frames, B * R, lay, d_out is not None)):
                L.paig_decoder_bwd(ptr(pvs) + 2 * D * 4, (R + 1) * 2 * D, 2 * D, R, ptr(tmpl), ptr(cont), ptr(bgp),
                                   *S["tgt_roll"], ptr(d_sse_roll), ptr(d_out), lay.frame, ptr(dpos_roll),
                                   ptr(slab) + nb_rec * slab_len * 4, ptr(scratch), B * R, roll_live, K, h, H, q)

        def dec_rec(q):    # reconstruction decoder backward: d enc_pos + partial source grads
            with self._p("dec_bwd:recon", 0, self._dec_bwd_bytes(F, F, lay, d_recons is not None)):
                L.paig_decoder_bwd(ptr(S["enc_pos"]), 0, 2 * K, 0, ptr(tmpl), ptr(cont), ptr(bgp), *x_view,
                                   ptr(d_sse_rec), ptr(d_recons), lay.frame, ptr(denc), ptr(slab), ptr(scratch), F, 0,
                                   K, h, H, q)

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
        self.linear_bwd(S["h1"], dh2, K * F, "encoder.l2", dh1, S["h1"], 1, st, ws, need_dx=not fused_l2)
        self.linear_bwd(S["l1_x"], dh1, K * F, "encoder.l1", dobjs, None, 0, st, ws)
        # every gradient of the flat buffer's early bucket is final (queued on
        # this stream): the data-parallel all-reduce of that bucket may start
        if hook and self.bucket_hook is not None:
            self.bucket_hook()

        # ---- mask softmax backward (incl. ReLU' of ShallowUNet's c13, Q13, and
        # the AvgPool2d backward of the UNet path)
        acts = S["acts"]
        dacts = {}
        if S.get("head_fused"):
            # fused c13 + softmax backward: c12's dY (ReLU' applied) and c13's
            # weight/bias partials (one slab row per block)
            c = lay.ops[-1]["src"][2]
            dX12 = _empty(F * c * HW, dev)
            nb = L.paig_head_mask_blocks(F, H, H)
            nw = K * c + K
            hs = _empty(nb * nw, dev)
            L.paig_head_mask_bwd(ptr(acts["A12"]), ptr(self.p(lay.prefix + "c13.weight")),
                                 ptr(self.p(lay.prefix + "c13.bias")), *x_view, ptr(S["masks"]), ptr(dobjs), ptr(dX12),
                                 ptr(hs), F, K, H, H, st)
            g13 = self.g(lay.prefix + "c13.weight")
            assert self.g(lay.prefix + "c13.bias").data_ptr() == g13.data_ptr() + K * c * 4, "c13 grads not contiguous"
            S["extra_slabs"].append((hs, nb, nw, g13))
            dacts["A12"] = dX12
        else:
            dLG = _empty(F * K * HW, dev)
            L.paig_mask_softmax_bwd(ptr(acts["LG"]), x_view[0], x_view[1], x_view[2], x_view[3], ptr(S["masks"]),
                                    ptr(dobjs), ptr(dLG), F, K, 3, H, H,
                                    (1 if lay.lg_relu else 0) | (2 if lay.unet else 0), st)
            dacts["LG"] = dLG
        self._unet_backward(S, dacts, st)

    def _fused_bwd(self, cin, cout, Hl, ks, cm):
        """The layer backward runs as one fused launch (paig_conv2d_bwd)
        where the library has the shape; PAIG_FUSED_BWD=0 keeps the separate
        data- and weight-gradient kernels (A/B)."""
        if os.environ.get("PAIG_FUSED_BWD", "1") == "0" or not cm:
            return False
        return bool(self.L.paig_conv2d_bwd_supported(cin, cout, Hl, Hl, ks, cm))

    @staticmethod
    def _check_fresh(S):
        if S.get("consumed"):
            raise PaigError("a second backward through one forward (retain_graph=True) is not supported: the "
                            "forward's saved state (activation maxima slots) was released by the first backward")

    def _unet_backward(self, S, dacts, st):
        self._check_fresh(S)
        lay = S["lay"]
        L = self.L
        dev = S["x"].device
        acts = S["acts"]
        view = S["view"]
        F, H = lay.F, lay.H
        fused = S.get("head_fused", False)
        # the fused head wrote c12's dY (dacts["A12"]); otherwise dLG is the start
        written = {"A12": [(0, lay.ops[-1]["src"][2])]} if fused else {"LG": [(0, lay.K)]}
        nops = len(lay.ops) - 1 if fused else len(lay.ops)
        cm = S["cm"]

        def dview(region):
            buf, off, n = region
            C, lvl = lay.bufs[buf]
            hw = (H // lvl) ** 2
            if buf not in dacts:
                dacts[buf] = _empty(F * C * hw, dev)
            t = dacts[buf]
            return (t.data_ptr() + off * hw * 4, C * hw), lvl

        def state(region):
            buf, off, n = region
            spans = written.get(buf, [])
            cov = sum(max(0, min(off + n, a + c) - max(off, a)) for a, c in spans)
            if cov == 0:
                return "write"
            if cov == n:
                return "accum"
            raise RuntimeError(f"partially written gradient region {region}")

        def mark(region):
            written.setdefault(region[0], []).append((region[1], region[2]))

        slabs = []
        folded_ups = set()   # upsample ops whose backward a fused conv backward did
        for i in range(nops - 1, -1, -1):
            if i in folded_ups:
                continue
            op = lay.ops[i]
            if op["op"] == "pool" and i in S.get("pcode", {}):
                continue   # folded into the pooled conv's backward (its dY staging), below
            fin = lay.fin[i]
            relu_fin = [r for r, relu in fin if relu]
            src, dst = op["src"], op["dst"]
            dyv, dlvl = dview(dst)
            if op["op"] == "conv":
                sv, slvl, xfl = S["conv_input"](i, op)
                Hl = H // slvl
                cin, cout, ks = src[2], dst[2], op["ks"]
                # weight + bias gradient: per-block partials, then one reduction
                nblk_max = 1024
                slab = _empty(nblk_max * (cout * cin * ks * ks + cout), dev)
                nb = ctypes.c_int(0)
                fl = 2 * F * cin * cout * ks * ks * Hl * Hl
                gw = self.g(lay.prefix + op["name"] + ".weight")
                n_w = cout * cin * ks * ks
                if xfl and self._fused_bwd(cin, cout, Hl, ks, cm | 32):
                    # fused-upsample input (c7 / c10): the layer backward AND the
                    # upsample's backward in one launch -- the data gradient of
                    # the upsampled tensor never reaches memory; the launch
                    # writes the half-resolution source's gradient
                    up = lay.fused_up[i]
                    ui = lay.ops.index(up)
                    usrc = up["src"]
                    dxv, _ = dview(usrc)
                    mode = state(usrc)
                    assert mode == "write", f"{op['name']}: upsample source gradient already written"
                    flags = cm | 32
                    aux = (None, 0)
                    if any(relu for r, relu in lay.fin[ui] if r == usrc):
                        a = view(usrc)[0]
                        aux = (a[0], a[1])
                        flags |= 2
                    nbytes = 4 * F * (cin * (Hl // 2) ** 2 * (2 if flags & 2 else 1) + cout * Hl * Hl)
                    with self._p("conv_bwd:" + op["name"], 2 * fl, nbytes):
                        L.paig_conv2d_bwd(sv[0], sv[1], sv[2], sv[3], dyv[0], dyv[1], dxv[0], dxv[1], aux[0], aux[1],
                                          ptr(self.p(lay.prefix + op["name"] + ".weight")), ptr(slab), nblk_max,
                                          ctypes.byref(nb), F, cin, cout, Hl, Hl, ks, flags, S["xmax"](i), XMAX_SLOTS,
                                          None, 0, None, 0, S["wprep"].get((i, 1)), st)
                    slabs.append((slab, nb.value, n_w + cout, gw))
                    mark(usrc)
                    folded_ups.add(ui)
                    continue
                if src[0] != "X0" and not xfl and self._fused_bwd(cin, cout, Hl, ks, cm):
                    # the layer's data and weight gradients in ONE launch from
                    # one staging of dY and X (csrc/conv_bwd.hip)
                    dxv, _ = dview(src)
                    mode = state(src)
                    flags = cm | (4 if mode == "accum" else 0)
                    aux = (None, 0)
                    if relu_fin:
                        assert len(fin) == 1 and fin[0][0] == src, f"{op['name']}: mixed ReLU finalization"
                        a = view(src)[0]
                        aux = (a[0], a[1])
                        flags |= 2
                    # algorithmic bytes: X and dY read, dX written (+ read when accumulating)
                    nbytes = 4 * F * Hl * Hl * (cin + cout + cin * (2 if mode == "accum" else 1))
                    # the max pool of this output (next op), folded: its
                    # gradient and window codes join the dY staging
                    fold = (None, 0, None, 0)
                    pj = i + 1
                    if pj in S.get("pcode", {}):
                        # the kernel reads this output's skip-path gradient
                        # (dY): its concat partner must have written it
                        assert state(dst) == "accum", f"{op['name']}: pool fold before the skip gradient (plan error)"
                        pdv, _ = dview(lay.ops[pj]["dst"])
                        cb, cfs = S["pcode"][pj]
                        fold = (pdv[0], pdv[1], cb.data_ptr(), cfs)
                        flags |= 64
                        nbytes += F * (4 * cout + cout) * (Hl // 2) ** 2   # pooled gradient + codes
                    with self._p("conv_bwd:" + op["name"], 2 * fl, nbytes):
                        L.paig_conv2d_bwd(sv[0], sv[1], sv[2], sv[3], dyv[0], dyv[1], dxv[0], dxv[1], aux[0], aux[1],
                                          ptr(self.p(lay.prefix + op["name"] + ".weight")), ptr(slab), nblk_max,
                                          ctypes.byref(nb), F, cin, cout, Hl, Hl, ks, cm | (flags & 70),
                                          S["xmax"](i), XMAX_SLOTS, *fold, S["wprep"].get((i, 1)), st)
                    slabs.append((slab, nb.value, n_w + cout, gw))
                    mark(src)
                    continue
                nbytes = 4 * F * (cin * (Hl // (2 if xfl else 1)) ** 2 + cout * Hl * Hl)
                with self._p("conv_wgrad:" + op["name"], fl, nbytes):
                    L.paig_conv2d_wgrad_ex(sv[0], sv[1], sv[2], sv[3], dyv[0], dyv[1], ptr(slab), nblk_max,
                                           ctypes.byref(nb), F, cin, cout, Hl, Hl, ks, xfl | cm, S["xmax"](i),
                                           XMAX_SLOTS, st)
                gb = self.g(lay.prefix + op["name"] + ".bias")
                assert gb.data_ptr() == gw.data_ptr() + n_w * 4, "flat grads: weight and bias must be adjacent"
                slabs.append((slab, nb.value, n_w + cout, gw))
                if src[0] == "X0":
                    continue
                dxv, _ = dview(src)
                mode = state(src)
                flags = 8 | (4 if mode == "accum" else 0)
                aux = (0, 0)
                if relu_fin:
                    assert len(fin) == 1 and fin[0][0] == src, f"{op['name']}: mixed ReLU finalization"
                    a = view(src)[0]
                    aux = (a[0], a[1])
                    flags |= 2
                W_ = self.p(lay.prefix + op["name"] + ".weight")
                nbytes = 4 * F * Hl * Hl * (cout + cin * (1 + (1 if flags & 2 else 0) + (1 if flags & 4 else 0)))
                with self._p("conv_dgrad:" + op["name"], fl, nbytes):
                    L.paig_conv2d_fwd_pw(dyv[0], dyv[1], 0, 0, dxv[0], dxv[1], aux[0] or None, aux[1], ptr(W_), None,
                                         F, cout, cin, Hl, Hl, ks, flags | cm, None, 0, None, 0,
                                         S["wprep"].get((i, 1)), st)
                mark(src)
            elif op["op"] == "pool":
                sv, slvl = view(src)
                Hl = H // slvl
                dxv, _ = dview(src)
                # the pool kernel accumulates into the concat partner's gradient
                assert state(src) == "accum", "maxpool backward reached before its concat partner (plan error)"
                relu = any(relu for r, relu in fin if r == src)
                assert relu, "pool sources are ReLU'd activations in both U-Nets"
                L.paig_maxpool2_bwd_relu(sv[0], sv[1], dyv[0], dyv[1], dxv[0], dxv[1], F, src[2], Hl, Hl, st)
                mark(src)
            else:
                sv, slvl = view(src)
                Hs, Ho = H // slvl, H // dlvl
                dxv, _ = dview(src)
                assert state(src) == "write"
                relu = any(relu for r, relu in fin if r == src)
                L.paig_upsample2_bwd(dyv[0], dyv[1], sv[0], sv[1], dxv[0], dxv[1], F, src[2], Hs, Hs, Ho, Ho,
                                     int(relu), st)
                mark(src)
        # all conv weight/bias gradients (+ the velocity MLP's): one batched
        # deterministic reduction
        slabs = slabs + S.get("extra_slabs", [])
        n = len(slabs)
        srcs = (ctypes.c_void_p * n)(*[ptr(s[0]) for s in slabs])
        nbs = (ctypes.c_int * n)(*[s[1] for s in slabs])
        lens = (ctypes.c_int * n)(*[s[2] for s in slabs])
        dsts = (ctypes.c_void_p * n)(*[ptr(s[3]) for s in slabs])
        L.paig_slab_reduce_multi(n, srcs, nbs, lens, dsts, 0, st)
        S["_slabs"] = slabs
        self._release_xmax(S)
