"""Flat parameter / gradient storage and the fused optimizers.

All live fp32 parameters of a PhysicsNet share ONE contiguous device buffer
(each nn.Parameter is a view into it, so state_dict keys, shapes and
load_state_dict are unchanged), and so do their gradients.  This makes the
data-parallel exchange one RCCL all-reduce of one buffer and the optimizer
one kernel launch (nn/network/base.py:12-17, :150-152 in the reference run a
per-parameter torch optimizer).  The 0-dim float64 physics parameters
(cells.py:28-29, 92-93; quirk Q9) get a tiny flat fp64 buffer of their own.
"""
import contextlib
import math
import weakref

import torch
import torch.distributed as dist

from ._lib import lib, ptr, stream_handle


# parameter (by id) -> (FlatParams, name): lets a standalone submodule call
# (nn/network/modules.py) deposit its gradients into the owning flat buffer
_OWNER = weakref.WeakValueDictionary()


class _DeferredMean:
    """An asynchronous gloo SUM all-reduce whose divide by the world size
    runs at wait(): the same start / overlap / wait() contract as RCCL's AVG
    work handle (FlatParams.allreduce_early / allreduce_grads)."""

    def __init__(self, work, t, n):
        self.work, self.t, self.n = work, t, n

    def wait(self):
        self.work.wait()
        self.t.div_(self.n)


def deposit_grad(p, g):
    """Add gradient g to parameter p with torch semantics (p.grad None ->
    set, else accumulate).  A parameter that lives in a FlatParams buffer gets
    it in its flat gradient slot (what FlatOptimizer and the DP all-reduce
    read); any other parameter gets p.grad directly."""
    fp = _OWNER.get(id(p))
    if fp is not None and fp.index and fp._params_by_id().get(id(p)) is not None:
        fp.deposit({fp._params_by_id()[id(p)]: g})
        return
    g = g.detach().reshape(p.shape).to(p.dtype)
    if p.grad is None:
        p.grad = g.clone()
    else:
        p.grad.add_(g)


class FlatParams:
    def __init__(self, model, names, early=()):
        self.model = model
        self.names = list(names)
        self.early = tuple(early)   # name prefixes of the early-final gradient bucket (a prefix of names)
        self.index = {}
        self.p32 = self.p64 = self.g32 = self.g64 = None
        self.device = None
        self._redirect = None
        self._early_work = None
        self.n32_early = 0

    def _params(self):
        pd = dict(self.model.named_parameters())
        return [(n, pd[n]) for n in self.names]

    def ensure(self):
        """(Re)build the flat buffers if any parameter moved (e.g. .to(device))."""
        if self.p32 is not None:
            ok = True
            for n, p in self._params():
                kind, off, num, _ = self.index[n]
                base = self.p32 if kind == 32 else self.p64
                if p.data_ptr() != base.data_ptr() + off * base.element_size() or p.device != base.device:
                    ok = False
                    break
            if ok:
                return False
        self.rebuild()
        return True

    def rebuild(self):
        params = self._params()
        dev = params[0][1].device
        n32 = sum(p.numel() for _, p in params if p.dtype == torch.float32)
        n64 = sum(p.numel() for _, p in params if p.dtype == torch.float64)
        self.p32 = torch.empty(n32, device=dev, dtype=torch.float32)
        self.p64 = torch.empty(max(n64, 1), device=dev, dtype=torch.float64)
        self.g32 = torch.zeros(n32, device=dev, dtype=torch.float32)
        self.g64 = torch.zeros(max(n64, 1), device=dev, dtype=torch.float64)
        o32 = o64 = 0
        self.index = {}
        with torch.no_grad():
            for n, p in params:
                num = p.numel()
                if p.dtype == torch.float32:
                    self.p32[o32:o32 + num].copy_(p.data.reshape(-1))
                    p.data = self.p32[o32:o32 + num].view(p.shape)
                    self.index[n] = (32, o32, num, tuple(p.shape))
                    o32 += num
                elif p.dtype == torch.float64:
                    self.p64[o64:o64 + num].copy_(p.data.reshape(-1))
                    p.data = self.p64[o64:o64 + num].view(p.shape)
                    self.index[n] = (64, o64, num, tuple(p.shape))
                    o64 += num
                else:
                    raise TypeError(f"{n}: unsupported dtype {p.dtype}")
        self.n32, self.n64 = n32, n64
        for n, p in params:
            _OWNER[id(p)] = self
        # the early bucket = the leading fp32 parameters named by self.early
        self.n32_early = 0
        for n, p in params:
            if p.dtype != torch.float32 or not n.startswith(self.early):
                break
            self.n32_early += p.numel()
        self.device = dev
        self._early_work = None
        return True

    def _params_by_id(self):
        return {id(p): n for n, p in self._params()}

    def deposit(self, grads):
        """{name: gradient tensor} into the flat gradient slots: copied where
        p.grad is None (and p.grad set to the slot view), added otherwise."""
        L = lib()
        pd = dict(self._params())
        for n, g in grads.items():
            kind, off, num, shape = self.index[n]
            base = self.g32 if kind == 32 else self.g64
            slot = base[off:off + num]
            g = g.detach().reshape(-1).to(base.dtype).contiguous()
            p = pd[n]
            if p.grad is None:
                slot.copy_(g)
                p.grad = slot.view(shape)
            elif kind == 32:
                L.paig_axpby(ptr(g), ptr(slot), num, 1.0, 1.0, stream_handle(slot.device))
            else:
                slot.add_(g)   # the 0-dim fp64 physics parameters

    @contextlib.contextmanager
    def partial_backward(self, prefixes):
        """A backward that writes only the parameters named by ``prefixes``
        (a standalone submodule call): the engine writes them into a zeroed
        redirect buffer, from which they are deposited with torch semantics;
        every other parameter's gradient is left as it was."""
        self.ensure()
        prefixes = tuple(prefixes)
        red = (torch.zeros_like(self.g32), torch.zeros_like(self.g64))
        self._redirect = red
        try:
            yield
        finally:
            self._redirect = None
        grads = {}
        for n, p in self._params():
            if n.startswith(prefixes):
                kind, off, num, shape = self.index[n]
                grads[n] = (red[0] if kind == 32 else red[1])[off:off + num]
        self.deposit(grads)

    def grad_view(self, name):
        kind, off, num, shape = self.index[name]
        g = self._redirect if self._redirect is not None else (self.g32, self.g64)
        base = g[0] if kind == 32 else g[1]
        return base[off:off + num].view(shape)

    # -- autograd integration ------------------------------------------------
    def begin_backward(self):
        """Returns True if gradients must accumulate (grads not zeroed since the
        last backward, the torch semantics the reference relies on)."""
        params = self._params()
        acc = any(p.grad is not None for _, p in params)
        if acc:
            self._redirect = (torch.empty_like(self.g32), torch.empty_like(self.g64))
            self._redirect[1].zero_()
            # a parameter whose grad is None gets this backward's gradient, not
            # that plus whatever its slot still holds from before zero_grad
            for n, p in params:
                if p.grad is None:
                    self.slot(n).zero_()
        return acc

    def slot(self, name):
        """The flat gradient slot of a parameter (1-D view)."""
        kind, off, num, _ = self.index[name]
        return (self.g32 if kind == 32 else self.g64)[off:off + num]

    def end_backward(self, accumulated, none_prefixes=()):
        if accumulated:
            L = lib()
            st = stream_handle(self.g32.device)
            L.paig_axpby(ptr(self._redirect[0]), ptr(self.g32), self.n32, 1.0, 1.0, st)
            if self.n64:
                self.g64.add_(self._redirect[1])  # 2 fp64 scalars
            self._redirect = None
        self.attach_grads(none_prefixes)

    def attach_grads(self, none_prefixes=()):
        """p.grad = its flat view; parameters the backward did not reach
        (name prefixes in none_prefixes) keep grad None unless they already
        had an accumulated gradient."""
        none_prefixes = tuple(none_prefixes)
        for n, p in self._params():
            if none_prefixes and n.startswith(none_prefixes) and p.grad is None:
                continue
            p.grad = self.grad_view(n)

    # tests only: run the data-parallel path (early-bucket all-reduce, late
    # bucket + fp64 scalars) in a world of one process, the only RCCL run a
    # one-GPU box allows (tests/test_gpu_dp.py::test_rccl_world1_step_bit_identical)
    FORCE_DP = False

    @staticmethod
    def _dp(group):
        return dist.is_available() and dist.is_initialized() and (dist.get_world_size(group) > 1 or
                                                                   FlatParams.FORCE_DP)

    @staticmethod
    def _mean(t, group, async_op=False):
        """In-place mean over the group: RCCL AVG over xGMI; gloo (the CPU
        harness of the DP path) has no AVG, so SUM then scale -- asynchronous
        too when asked (the divide deferred to wait()), so the early-bucket
        start / overlap / wait ordering runs the same way on both backends."""
        if dist.get_backend(group) == "nccl":
            return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group, async_op=async_op)
        n = dist.get_world_size(group)
        if async_op:
            return _DeferredMean(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True), t, n)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(n)
        return None

    def allreduce_early(self, group=None):
        """Start the mean all-reduce of the early-final bucket (asynchronous
        on RCCL: it runs on the process group's stream, ordered after the
        gradient kernels already queued, while the U-Net backward proceeds).
        A no-op while gradients accumulate into a redirect buffer."""
        if not self._dp(group) or self._redirect is not None or self.n32_early == 0 or self._early_work is not None:
            return
        self._early_work = (self._mean(self.g32[:self.n32_early], group, async_op=True), group)

    def allreduce_grads(self, group=None):
        """Mean of the gradients over the data-parallel group (RCCL over xGMI):
        the late bucket (+ the fp64 scalars) now, the early bucket unless
        allreduce_early already started it, whose completion is then awaited."""
        if not self._dp(group):
            self._early_work = None
            return
        started = self._early_work is not None
        lo = self.n32_early if started else 0
        if lo < self.n32:
            self._mean(self.g32[lo:], group)
        if self.n64:
            self._mean(self.g64, group)
        if started:
            self._early_work[0].wait()
            self._early_work = None


class FlatOptimizer:
    """Drop-in for the reference's torch optimizers (OPTIMIZERS, base.py:12-17)
    acting on the flat buffers with one fused HIP kernel per dtype.

    Exposes param_groups/zero_grad/step/state_dict like torch.optim, and
    performs the data-parallel gradient all-reduce before the update when a
    process group is initialised (the reference is single-GPU)."""

    def __init__(self, model, kind, lr, **hp):
        self.model = model
        self.kind = kind
        self.param_groups = [{"params": [p for _, p in model._flat._params()], "lr": lr, **hp}]
        self.hp = hp
        self.state = {}
        self.steps = 0        # steps taken by every parameter (the fused path)
        self._psteps = None   # per-parameter steps once a step skipped some (grad None), as torch counts them
        self._bufs = None

    def _ensure_state(self):
        flat = self.model._flat
        if self._bufs is None or self._bufs[0].numel() != flat.n32 or self._bufs[0].device != flat.p32.device:
            z32 = lambda: torch.zeros(flat.n32, device=flat.p32.device)  # noqa: E731
            z64 = lambda: torch.zeros(max(flat.n64, 1), device=flat.p32.device, dtype=torch.float64)  # noqa: E731
            if self.kind == "adam":
                self._bufs = (z32(), z32(), z64(), z64())
            else:
                self._bufs = (z32(), z64())
            self.steps = 0
            self._psteps = None

    def zero_grad(self, set_to_none=True):
        for _, p in self.model._flat._params():
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    @torch.no_grad()
    def step(self, closure=None):
        flat = self.model._flat
        flat.ensure()
        self._ensure_state()
        flat.allreduce_grads()
        params = flat._params()
        have = [p.grad is not None for _, p in params]
        if all(have) and self._psteps is None:
            # every parameter has a gradient and the same step count: one
            # fused launch per dtype over the whole flat buffers
            self.steps += 1
            if self.kind == "rmsprop":   # both dtypes in one launch
                a, eps = self.hp.get("alpha", 0.99), self.hp.get("eps", 1e-8)
                lib().paig_rmsprop_mixed(ptr(flat.p32), ptr(flat.g32), ptr(self._bufs[0]), flat.n32, ptr(flat.p64),
                                         ptr(flat.g64), ptr(self._bufs[1]) if flat.n64 else None, flat.n64,
                                         float(self.param_groups[0]["lr"]), a, eps, stream_handle(flat.p32.device))
                return None
            self._launch(32, 0, flat.n32, self.steps)
            if flat.n64:
                self._launch(64, 0, flat.n64, self.steps)
            return None
        # torch semantics: a parameter whose grad is None is skipped (no
        # update, no state change, no step count)
        if self._psteps is None:
            self._psteps = {n: self.steps for n, _ in params}
        for (n, _), h in zip(params, have):
            if h:
                self._psteps[n] += 1
                kind, off, num, _ = flat.index[n]
                self._launch(kind, off, num, self._psteps[n])
        if len(set(self._psteps.values())) == 1:   # back in lockstep: the fused path again
            self.steps = next(iter(self._psteps.values()))
            self._psteps = None
        return None

    def _launch(self, kind, off, num, step):
        """The update of flat elements [off, off + num) of one dtype."""
        flat = self.model._flat
        L = lib()
        st = stream_handle(flat.p32.device)
        lr = float(self.param_groups[0]["lr"])
        e32, e64 = 4 * off, 8 * off

        def at(t, e):
            return ptr(t) + e if t is not None else None

        if self.kind == "rmsprop":
            a, eps = self.hp.get("alpha", 0.99), self.hp.get("eps", 1e-8)
            # one launch for both dtypes when called for the whole buffers
            # (fp32 hyper-parameters rounded as torch's fp32 math does)
            if kind == 32:
                L.paig_rmsprop_mixed(at(flat.p32, e32), at(flat.g32, e32), at(self._bufs[0], e32), num, None, None,
                                     None, 0, lr, a, eps, st)
            else:
                L.paig_rmsprop_mixed(None, None, None, 0, at(flat.p64, e64), at(flat.g64, e64), at(self._bufs[1], e64),
                                     num, lr, a, eps, st)
        elif self.kind == "adam":
            b1, b2 = self.hp.get("betas", (0.9, 0.999))
            eps = self.hp.get("eps", 1e-8)
            bc1 = 1 - b1 ** step
            bc2s = math.sqrt(1 - b2 ** step)
            if kind == 32:
                L.paig_adam_f32(at(flat.p32, e32), at(flat.g32, e32), at(self._bufs[0], e32), at(self._bufs[1], e32),
                                num, lr, b1, b2, eps, bc1, bc2s, st)
            else:
                L.paig_adam_f64(at(flat.p64, e64), at(flat.g64, e64), at(self._bufs[2], e64), at(self._bufs[3], e64),
                                num, lr, b1, b2, eps, bc1, bc2s, st)
        else:  # sgd / momentum
            mom = self.hp.get("momentum", 0.0)
            first = int(step == 1)
            if kind == 32:
                L.paig_sgd_f32(at(flat.p32, e32), at(flat.g32, e32), at(self._bufs[0], e32) if mom else None, num, lr,
                               mom, first, st)
            else:
                L.paig_sgd_f64(at(flat.p64, e64), at(flat.g64, e64), at(self._bufs[1], e64) if mom else None, num, lr,
                               mom, first, st)

    def state_dict(self):
        return {"kind": self.kind, "steps": self.steps, "psteps": None if self._psteps is None else dict(self._psteps),
                "param_groups": [
            {k: v for k, v in g.items() if k != "params"} for g in self.param_groups],
            "bufs": [b.detach().cpu() for b in (self._bufs or ())]}

    def load_state_dict(self, sd):
        self.steps = sd["steps"]
        self._psteps = dict(sd["psteps"]) if sd.get("psteps") else None
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)
        if sd.get("bufs"):
            dev = self.model._flat.p32.device
            self._bufs = tuple(b.to(dev) for b in sd["bufs"])
