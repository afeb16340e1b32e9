"""One training step of the reference loop body (nn/network/base.py:141-152:
forward, compute_loss, zero_grad, backward, optimizer.step) captured as HIP
graph replays on a fixed input buffer — the form bench.py times and the
data-parallel test drives.

  * N = 1: forward + loss + backward (+ the RMSprop launch, which has no
    step-dependent scalar) in ONE graph;
  * N > 1 (split): two graphs cut where the early gradient bucket is final
    (Engine.bucket_hook); between the replays that bucket's all-reduce
    starts (FlatParams.allreduce_early), overlapping the U-Net backward of
    the second replay; FlatOptimizer.step then reduces the late bucket and
    the fp64 scalars and applies the update eagerly.
"""
import torch


class GraphStep:
    def __init__(self, model, xbuf, world=1, split=None, graph=True, optimizer_in_graph=True):
        """Call eager() for warm-up steps, then capture() (when graph)."""
        self.m = model
        self.xbuf = xbuf
        self.world = world
        self.use_graph = graph
        self.split = bool(graph and (world > 1 if split is None else split))
        self.opt_in_graph = bool(graph and optimizer_in_graph and world == 1 and not self.split
                                 and model.optimizer.kind == "rmsprop")
        self.eng = model._native()
        self.one = None
        self.graph = None
        self.replays = 0

    def body(self, x):
        m = self.m
        m.output = m(x)
        loss, _ = m.compute_loss()
        m.optimizer.zero_grad(set_to_none=True)
        # d loss / d loss = 1 from a persistent tensor (made before any graph
        # capture): autograd's implicit ones_like would be a fill kernel per step
        if self.one is None:
            self.one = torch.ones_like(loss)
        loss.backward(self.one)
        return loss

    def eager(self):
        loss = self.body(self.xbuf)
        self.m.optimizer.step()
        return loss

    def capture(self):
        if not self.use_graph:
            return
        m, eng = self.m, self.eng
        if self.one is None:   # the seed gradient must exist before any capture
            self.one = torch.ones((), device=self.xbuf.device)
        torch.cuda.synchronize()
        if not self.split:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                lg = self.body(self.xbuf)
                if self.opt_in_graph:
                    m.optimizer.step()
            self.graph = ((g,), lg)
        else:
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            seen = []

            def cut():   # engine.bucket_hook: the early bucket is final here
                g1.capture_end()
                g2.capture_begin(pool=g1.pool(), capture_error_mode="relaxed")
                seen.append(1)

            cap = torch.cuda.Stream()
            cap.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cap):
                # relaxed: the cut runs on the autograd engine's device thread
                g1.capture_begin(capture_error_mode="relaxed")
                eng.bucket_hook = cut
                try:
                    lg = self.body(self.xbuf)
                finally:
                    eng.bucket_hook = m._flat.allreduce_early
                g2.capture_end()
            torch.cuda.current_stream().wait_stream(cap)
            assert seen == [1], "backward did not reach the bucket split point"
            self.graph = ((g1, g2), lg)
        torch.cuda.synchronize()

    def __call__(self):
        if self.graph is None:
            return self.eager()
        gs, lg = self.graph
        self.replays += 1
        gs[0].replay()
        if len(gs) == 2:
            self.m._flat.allreduce_early()   # overlaps the second graph (U-Net backward)
            gs[1].replay()
        if not self.opt_in_graph:
            self.m.optimizer.step()
        return lg

    def finish(self):
        """The captured RMSprop step ran Python once, at capture: count its
        replays in the optimizer's step counter (RMSprop's update does not
        depend on it)."""
        if self.opt_in_graph:
            self.m.optimizer.steps += self.replays
            self.replays = 0
