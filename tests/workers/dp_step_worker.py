"""Child process of tests/test_gpu_dp.py (not collected by pytest): one rank
of the data-parallel training step on cuda:0 over gloo, or the
single-process reference on the concatenated batch.

  python tests/workers/dp_step_worker.py --mode dp --rank R --world 2 --port P --kind K --out DIR
  python tests/workers/dp_step_worker.py --mode single --kind K --out DIR

Both run the same 3 steps (3 fixed global batches of 2B sequences,
synthetic spring_color, seq 12) through paig_reproduction_amd.graph_step
(bench.py's step): DP ranks take disjoint halves of every global batch and
replay the split HIP graph with the early-bucket all-reduce between the two
replays, then FlatOptimizer.step (late bucket + fp64 scalars, the update).
Writes the flat gradient buffer after every step and the final parameters
(rank 0 / single) to DIR as .npy.
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
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    world = a.world if a.mode == "dp" else 1
    if a.mode == "dp":
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(a.port)
        dist.init_process_group("gloo", rank=a.rank, world_size=world)
    from paig_reproduction_amd.graph_step import GraphStep
    from paig_reproduction_amd.nn.datasets.synth import as_model_input, render_sequences
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet

    torch.manual_seed(0)
    m = PhysicsNet("spring_color", 100, 1, "spring_ode_cell", SEQ, 4, 6, 3.0, False, True, 32 * 32,
                   "conv_encoder", "conv_st_decoder", device=dev).to(dev)
    opt = {"momentum": "momentum", "rmsprop": "rmsprop"}[a.kind]
    m.build_optimizer(1e-3, opt, True)
    if world > 1:
        for t in m.state_dict().values():
            dist.broadcast(t, 0)
    # 3 global batches of 2 * B_RANK sequences (identical in every process)
    u8 = render_sequences("spring_color", 2 * B_RANK * STEPS, SEQ, seed=11)
    xs = torch.from_numpy(as_model_input(u8)).view(STEPS, 2 * B_RANK, SEQ, 3, 32, 32)
    nb = B_RANK if world > 1 else 2 * B_RANK
    xbuf = torch.empty((nb, SEQ, 3, 32, 32), device=dev)
    step = GraphStep(m, xbuf, world, graph=True)
    if world > 1:
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
        m.load_state_dict(init)
    m.build_optimizer(1e-3, opt, True)   # fresh optimizer state (the graph reads the same flat buffers)
    torch.cuda.synchronize()
    flat = m._flat
    for i in range(STEPS):
        load(i)
        step()
        torch.cuda.synchronize()
        if a.mode == "single" or a.rank == 0:
            np.save(os.path.join(a.out, f"g32_{i}.npy"), flat.g32.cpu().numpy())
            np.save(os.path.join(a.out, f"g64_{i}.npy"), flat.g64.cpu().numpy())
    if a.mode == "single" or a.rank == 0:
        np.save(os.path.join(a.out, "p32.npy"), flat.p32.cpu().numpy())
        np.save(os.path.join(a.out, "p64.npy"), flat.p64.cpu().numpy())
    if world > 1:
        # every rank holds the same parameters
        t = flat.p32.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert torch.equal(t, flat.p32), "ranks diverged"
        dist.destroy_process_group()
    print("WORKER_OK", a.mode, a.rank, flush=True)


if __name__ == "__main__":
    main()
