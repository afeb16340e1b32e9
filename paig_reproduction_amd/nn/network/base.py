"""BaseNetTorch: the reference's trainer surface (nn/network/base.py:20-218),
same methods, arguments and side effects, driving the HIP step.

Differences (documented in DESIGN.md):
  * OPTIMIZERS map to FlatOptimizer (one fused HIP kernel over the flat
    parameter buffer) with the torch defaults the reference uses;
  * ``loss_mode`` (default "fresh"): the loss is taken on the CURRENT forward
    (the north star's combined loss).  "reference" reproduces quirk Q1: the
    train step's loss reads the stale ``self.output`` of the last eval batch;
  * when torch.distributed is initialised, the optimizer step first averages
    the flat gradient over the group (RCCL), and each rank trains on its own
    shard of every epoch (DataIterator(rank, world)).  The reference has no
    data parallelism, so its file side effects are made rank-safe here: rank 0
    alone deletes / creates save_dir, writes log.txt, code.zip, model.ckpt and
    outputs.npz, with barriers where other ranks read them; eval metrics are
    example-weighted means over all ranks (one all-reduce), and a set too small
    for the reference's batch (Q15: < 100 examples, one whole-set batch) is
    split into one near-equal share per rank instead.
"""
import logging
import os
import shutil
import sys

import numpy as np
import torch

from paig_reproduction_amd.flat import FlatOptimizer
from paig_reproduction_amd.nn.utils.misc import log_metrics, zipdir

logger = logging.getLogger("torch")
root_path = os.path.join(os.path.dirname(os.path.realpath(__file__)), "..", "..")

OPTIMIZERS = {
    "adam": lambda model, lr: FlatOptimizer(model, "adam", lr),
    "rmsprop": lambda model, lr: FlatOptimizer(model, "rmsprop", lr),
    "momentum": lambda model, lr: FlatOptimizer(model, "sgd", lr, momentum=0.9),
    "sgd": lambda model, lr: FlatOptimizer(model, "sgd", lr),
}


def _dp():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _rank():
    import torch.distributed as dist
    return dist.get_rank() if _dp() else 0


def _barrier():
    if _dp():
        import torch.distributed as dist
        dist.barrier()


class BaseNetTorch(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.train_metrics = {}
        self.eval_metrics = {}
        self.extra_train_fns = []
        self.extra_valid_fns = []
        self.extra_test_fns = []

    def run_extra_fns(self, type):
        if type == "train":
            extra_fns = self.extra_train_fns
        elif type == "valid":
            extra_fns = self.extra_valid_fns
        else:
            extra_fns = self.extra_test_fns
        for fn, args, kwargs in extra_fns:
            fn(*args, **kwargs)

    def conv_feedforward(self, inp):
        raise NotImplementedError

    def compute_loss(self):
        raise NotImplementedError

    def get_data(self, data_iterators):
        self.train_iterator, self.valid_iterator, self.test_iterator = data_iterators

    def get_batch(self, batch_size, iterator):
        batch_x, batch_y = iterator.next_batch(batch_size)
        if batch_y is None:
            feed_dict = {"input": batch_x}
        else:
            feed_dict = {"input": batch_x, "target": batch_y}
        return feed_dict, (batch_x, batch_y)

    def initialize_graph(self, save_dir, use_ckpt, ckpt_dir=""):
        """nn/network/base.py:65-94, including Q14 (an existing save_dir is
        deleted unless use_ckpt).  Data-parallel: every rank decides from what
        existed before any rank touched the directory; rank 0 alone deletes /
        creates it; the checkpoint is read after a barrier."""
        self.save_dir = save_dir
        existed = os.path.exists(save_dir)
        _barrier()   # every rank has looked before rank 0 changes anything
        rank0 = _rank() == 0
        if existed:
            if use_ckpt:
                restore = True
                restore_dir = ckpt_dir if ckpt_dir else save_dir
            else:
                if rank0:
                    logger.info("Folder exists, deleting...")
                    shutil.rmtree(save_dir)
                    os.makedirs(save_dir)
                restore = False
        else:
            if rank0:
                os.makedirs(save_dir)
            if use_ckpt:
                restore = True
                restore_dir = ckpt_dir
            else:
                restore = False
        _barrier()
        if restore:
            print(f"Loading model from: {restore_dir + '/model.ckpt'}")
            sd = torch.load(os.path.join(restore_dir, "model.ckpt"), map_location=self.device, weights_only=True)
            self.load_state_dict(sd)

    def get_iterator(self, type):
        if type == "train":
            return self.train_iterator
        if type == "valid":
            return self.valid_iterator
        if type == "test":
            return self.test_iterator

    def add_train_logger(self):
        if _rank() != 0:   # one writer of log.txt
            return
        log_path = os.path.join(self.save_dir, "log.txt")
        fh = logging.FileHandler(log_path)
        fh.setFormatter(logging.Formatter('%(asctime)s - %(name)s - %(message)s'))
        logger.addHandler(fh)

    def _to_device(self, batch, requires_grad):
        t = torch.as_tensor(batch, device=self.device)
        if t.dtype != torch.float32:
            t = t.float()
        # the reference creates the input with requires_grad=True (Q10); its
        # gradient is never used, so it is not computed here.
        return t

    def train_model(self, epochs, batch_size, save_every_n_epochs, eval_every_n_epochs, print_interval, debug=False):
        """nn/network/base.py:112-172."""
        self.train()
        self.batch_size = batch_size
        self.add_train_logger()
        if _rank() == 0:
            zipdir(root_path, self.save_dir)
        logger.info("\n".join(sys.argv))
        step = 0
        if not debug and epochs > 0:
            valid_metrics_results = self.eval_performance(batch_size, type='valid')
            log_metrics(logger, "valid - epoch=%s" % 0, valid_metrics_results)

        for ep in range(1, epochs + 1):
            if self.anneal_lr:
                if ep == int(0.75 * epochs):
                    self.lr = self.lr / 5          # Q6: never reaches the optimizer
            while self.train_iterator.epochs_completed < ep:
                feed_dict, _ = self.get_batch(batch_size, self.train_iterator)
                inp = self._to_device(feed_dict["input"], True)
                result_sequence = self.forward(inp)
                if getattr(self, "loss_mode", "fresh") == "fresh":
                    self.output = result_sequence
                self.train_loss, self.eval_losses = self.compute_loss()
                self.train_metrics["train_loss"] = self.train_loss
                self.eval_metrics["eval_pred_loss"] = self.eval_losses[0]
                self.eval_metrics["eval_extrap_loss"] = self.eval_losses[1]
                self.eval_metrics["eval_recons_loss"] = self.eval_losses[2]
                self.loss = self.train_loss
                self.optimizer.zero_grad(set_to_none=True)
                if getattr(self, "_seed_grad", None) is None or self._seed_grad.shape != self.loss.shape:
                    self._seed_grad = torch.ones_like(self.loss)   # reused: no fill kernel per step
                self.loss.backward(self._seed_grad)
                self.optimizer.step()
                self.run_extra_fns("train")
                if step % print_interval == 0:
                    log_metrics(logger, "train - iter=%s" % step, self.train_metrics)
                    if hasattr(self, "check_numerics"):
                        self.check_numerics()
                step += 1

            if ep % eval_every_n_epochs == 0:
                print("eval running")
                valid_metrics_results = self.eval_performance(batch_size, type='valid')
                log_metrics(logger, "valid - epoch=%s" % ep, valid_metrics_results)

            if ep % save_every_n_epochs == 0:
                print("saving")
                if self._is_rank0():
                    torch.save(self.state_dict(), os.path.join(self.save_dir, "model.ckpt"))
                _barrier()   # the file is complete before any rank may restore it

        test_metrics_results = self.eval_performance(batch_size, type='test')
        log_metrics(logger, "test - epoch=%s" % epochs, test_metrics_results)

    @staticmethod
    def _is_rank0():
        return _rank() == 0

    def _reduce_metrics(self, per_batch, counts):
        """Example-weighted mean of the per-batch metric values over all
        batches of all ranks (the reference's np.mean over equal-size batches;
        exact for the uneven shares of a small set too)."""
        keys = list(per_batch)
        local = [sum(float(np.asarray(v).reshape(-1)[0]) * n for v, n in zip(per_batch[k], counts)) for k in keys]
        t = torch.tensor(local + [float(sum(counts))], dtype=torch.float64, device=self.device)
        if _dp():
            import torch.distributed as dist
            dist.all_reduce(t)
        t = t.cpu().numpy()
        return {k: np.float64(t[i] / max(t[-1], 1.0)) for i, k in enumerate(keys)}

    def eval_performance(self, batch_size, type='valid'):
        """nn/network/base.py:174-218 (Q15: whole set when it has < 100 examples)."""
        self.eval()
        with torch.no_grad():
            self.eval_metrics["eval_pred_loss"] = torch.tensor([0], device=self.device)
            self.eval_metrics["eval_extrap_loss"] = torch.tensor([0], device=self.device)
            self.eval_metrics["eval_recons_loss"] = torch.tensor([0], device=self.device)
            eval_metrics_results = {k: [] for k in self.eval_metrics.keys()}
            eval_outputs = {"input": [], "output": []}
            eval_iterator = self.get_iterator(type)
            eval_iterator.reset_epoch()
            counts = []
            while eval_iterator.get_epoch() < 1:
                if eval_iterator.X.shape[0] < 100:
                    # Q15: the whole set as one batch; data-parallel: one
                    # near-equal share of it per rank
                    n, w = eval_iterator.X.shape[0], max(getattr(eval_iterator, "world", 1), 1)
                    batch_size = -(-n // w)
                feed_dict, _ = self.get_batch(batch_size, eval_iterator)
                if len(feed_dict["input"]) == 0:   # more ranks than examples: nothing to evaluate here
                    continue
                counts.append(len(feed_dict["input"]))
                inp = self._to_device(feed_dict["input"], False)
                self.output = self.conv_feedforward(inp)
                self.train_loss, self.eval_losses = self.compute_loss()
                self.train_metrics["train_loss"] = self.train_loss
                self.eval_metrics["eval_pred_loss"] = self.eval_losses[0]
                self.eval_metrics["eval_extrap_loss"] = self.eval_losses[1]
                self.eval_metrics["eval_recons_loss"] = self.eval_losses[2]
                self.loss = self.train_loss
                for k in self.eval_metrics.keys():
                    eval_metrics_results[k].append(self.eval_metrics[k])
                fi = feed_dict["input"]
                eval_outputs["input"].append(fi.detach().cpu().numpy() if torch.is_tensor(fi) else fi)
                eval_outputs["output"].append(self.eval_losses)
            if _dp():
                eval_metrics_results = self._reduce_metrics(
                    {k: [i.detach().cpu().numpy() for i in v] for k, v in eval_metrics_results.items()}, counts)
            else:
                eval_metrics_results = {k: np.mean([i.detach().cpu().numpy() for i in v], axis=0)
                                        for k, v in eval_metrics_results.items()}
            ins = [np.asarray(a) for a in eval_outputs["input"]]
            outs = [[o.detach().cpu().numpy() for o in out] for out in eval_outputs["output"]]
            if _dp():   # every rank's inputs and per-batch losses, in rank order
                import torch.distributed as dist
                got = [None] * dist.get_world_size() if self._is_rank0() else None
                dist.gather_object((ins, outs), got, dst=0)
                if self._is_rank0():
                    ins = [a for g in got for a in g[0]]
                    outs = [o for g in got for o in g[1]]
            if self._is_rank0() and ins:
                np.savez_compressed(os.path.join(self.save_dir, "outputs.npz"),
                                    input=np.concatenate(ins, axis=0), output=np.array(outs))
            self.run_extra_fns(type)
            return eval_metrics_results
