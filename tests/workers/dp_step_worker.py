"""Child process of tests/test_gpu_dp.py (not collected by pytest): one rank
of the data-parallel training step on cuda:0 over gloo, or the
single-process reference on the concatenated batch.

  python tests/workers/dp_step_worker.py --mode dp --rank R --world 2 --port P --kind K --out DIR
  python tests/workers/dp_step_worker.py --mode single --kind K --out DIR --src DPDIR
  python tests/workers/dp_step_worker.py --mode dp --world 1 --backend nccl --force_dp --kind K --out DIR

The last form runs the data-parallel path (split graph, RCCL all-reduce of
the early bucket between the replays, FlatOptimizer.step with the late
bucket and the fp64 scalars) in a world of one process: RCCL's AVG over one
rank must leave every gradient and parameter bit-identical to the
single-process step.

Both run 3 steps (3 fixed global batches of 2B sequences, synthetic
spring_color, seq 12) through paig_reproduction_amd.graph_step (bench.py's
step): DP ranks take disjoint halves of every global batch and replay the
split HIP graph with the early-bucket all-reduce between the two replays,
then FlatOptimizer.step (late bucket + fp64 scalars, the update).  Rank 0
writes, per step, the state it started from (parameters, optimizer
buffers), the all-reduced flat gradients and the parameters after the
update.  The single-process run loads each of those starting states and
takes the same step on the whole batch, writing its gradients and updated
parameters: every step is compared from the same state (a multi-step
trajectory would part at the first near-tie max-pool / ReLU decision that a
one-ulp parameter difference flips).
"""
import argparse
import os
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B_RANK, SEQ, STEPS = 8, 12, 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["dp", "single"], required=True)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--kind", default="momentum")
    ap.add_argument("--out", required=True)
    ap.add_argument("--src", default="", help="single mode: the DP run's output directory")
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--force_dp", action="store_true", help="the DP path at world 1 (FlatParams.FORCE_DP)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    world = a.world if a.mode == "dp" else 1
    if a.mode == "dp":
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(a.port)
        dist.init_process_group(a.backend, rank=a.rank, world_size=world)
    from paig_reproduction_amd.flat import FlatParams
    from paig_reproduction_amd.graph_step import GraphStep
    FlatParams.FORCE_DP = a.force_dp
    from paig_reproduction_amd.nn.datasets.synth import as_model_input, render_sequences
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet

    torch.manual_seed(0)
    m = PhysicsNet("spring_color", 100, 1, "spring_ode_cell", SEQ, 4, 6, 3.0, False, True, 32 * 32,
                   "conv_encoder", "conv_st_decoder", device=dev).to(dev)
    m.build_optimizer(1e-3, a.kind, True)
    if world > 1:
        for t in m.state_dict().values():
            dist.broadcast(t, 0)
    # 3 global batches of 2 * B_RANK sequences (identical in every process)
    u8 = render_sequences("spring_color", 2 * B_RANK * STEPS, SEQ, seed=11)
    xs = torch.from_numpy(as_model_input(u8)).view(STEPS, 2 * B_RANK, SEQ, 3, 32, 32)
    nb = B_RANK if world > 1 else 2 * B_RANK
    xbuf = torch.empty((nb, SEQ, 3, 32, 32), device=dev)
    step = GraphStep(m, xbuf, world, graph=True, split=True if a.force_dp else None)
    if world > 1 or a.force_dp:
        assert step.split, "the DP step must use the split graph"
    # warm-up on the first batch, then capture; re-initialise the parameters
    # and optimizer state afterwards so the 3 timed steps start from the same point
    init = {k: v.detach().clone() for k, v in m.state_dict().items()}

    def load(i):
        x = xs[i]
        if world > 1:
            x = x[a.rank * B_RANK:(a.rank + 1) * B_RANK]
        xbuf.copy_(x.to(dev))

    load(0)
    step.eager()
    step.capture()
    with torch.no_grad():
        m.load_state_dict(init)   # in place: the captured graph reads the same flat buffers
    opt = m.optimizer
    opt._ensure_state()
    for b in opt._bufs:   # fresh optimizer state, in place (a captured RMSprop step reads these buffers)
        b.zero_()
    opt.steps = 0
    torch.cuda.synchronize()
    flat = m._flat
    save = a.mode == "single" or a.rank == 0

    def dump(tag, i, arrs):
        for nm, t in arrs.items():
            np.save(os.path.join(a.out, f"{tag}_{nm}_{i}.npy"), t.detach().cpu().numpy())

    for i in range(STEPS):
        if a.mode == "single":
            # start from the DP run's state before its step i
            src = a.src
            with torch.no_grad():
                flat.p32.copy_(torch.from_numpy(np.load(os.path.join(src, f"pre_p32_{i}.npy"))).to(dev))
                flat.p64.copy_(torch.from_numpy(np.load(os.path.join(src, f"pre_p64_{i}.npy"))).to(dev))
                for j, b in enumerate(opt._bufs):
                    b.copy_(torch.from_numpy(np.load(os.path.join(src, f"pre_buf{j}_{i}.npy"))).to(dev))
            opt.steps = i
        elif save:
            dump("pre", i, {"p32": flat.p32, "p64": flat.p64, **{f"buf{j}": b for j, b in enumerate(opt._bufs)}})
        load(i)
        step()
        torch.cuda.synchronize()
        if save:
            dump("post", i, {"g32": flat.g32, "g64": flat.g64, "p32": flat.p32, "p64": flat.p64})
    if a.mode == "dp" and world == 1:
        dist.destroy_process_group()
    if world > 1:
        # every rank holds the same parameters
        t = flat.p32.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert torch.equal(t, flat.p32), "ranks diverged"
        dist.destroy_process_group()
    print("WORKER_OK", a.mode, a.rank, flush=True)


if __name__ == "__main__":
    main()
