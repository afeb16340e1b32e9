"""Data-parallel path on CPU: world_size 2 over gloo (the GPU runs use RCCL).

Checks, per rank, the pieces the N-GPU bench relies on:
  * DataIterator(rank, world) hands each rank a disjoint shard of every epoch
    of a shared permutation (drop-last per global batch);
  * FlatParams.allreduce_grads averages the ONE flat gradient buffer, also
    when its early-final bucket was started ahead (allreduce_early);
  * the averaged per-rank gradients of the oracle step equal the gradient of
    the concatenated batch (the reference's losses are batch means, so equal
    per-rank batches make DP exact) -- the contract weak scaling depends on.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from paig_reproduction_amd.nn.datasets.iterators import DataIterator
        from paig_reproduction_amd.nn.network.physics_models import PhysicsNet
        from helpers import load_golden, golden_weights
        from oracle import physics_oracle as O

        # 1) sharded iterator
        X = np.arange(20, dtype=np.float32).reshape(20, 1)
        it = DataIterator(X, seed=3, rank=rank, world=world)
        mine = []
        while it.get_epoch() < 1:
            bx, _ = it.next_batch(3)
            mine.append(bx[:, 0].astype(int).tolist())
        allb = [None] * world
        dist.all_gather_object(allb, mine)
        for step in zip(*allb):
            flat = sum(step, [])
            assert len(set(flat)) == len(flat), "ranks overlap within a global batch"

        # 2) flat all-reduce (average) of the flat gradient buffer
        torch.manual_seed(0)
        m = PhysicsNet("spring_color", 100, 1, "spring_ode_cell", 12, 4, 6, 3.0, False, True, 32 * 32, "", "conv_st_decoder")
        flat = m._flat
        flat.rebuild()
        flat.g32.fill_(float(rank + 1))
        flat.g64.fill_(float(10 * (rank + 1)))
        flat.allreduce_grads()
        assert torch.allclose(flat.g32, torch.full_like(flat.g32, 1.5))
        assert torch.allclose(flat.g64, torch.full_like(flat.g64, 15.0))

        # 2b) bucketed exchange: the early-final bucket (VariableFromNetwork +
        # localiser l1/l2, leading the flat buffer) is reduced first, the rest
        # after the U-Net backward; the result is the same mean
        assert 0 < flat.n32_early < flat.n32
        for n in flat.names:
            kind, off, num, _ = flat.index[n]
            early = n.startswith(m.EARLY_GRADS)
            assert kind != 32 or early == (off + num <= flat.n32_early), n
        assert flat.n32_early / flat.n32 > 0.9   # most gradient bytes overlap the U-Net backward
        flat.g32.copy_(torch.arange(flat.n32, dtype=torch.float32) * (rank + 1))
        flat.g64.fill_(float(rank))
        flat.allreduce_early()
        flat.g32[flat.n32_early:].mul_(1.0)   # the late bucket is still being written here
        flat.allreduce_grads()
        assert torch.allclose(flat.g32, torch.arange(flat.n32, dtype=torch.float32) * 1.5)
        assert torch.allclose(flat.g64, torch.full_like(flat.g64, 0.5))
        assert flat._early_work is None

        # 3) DP equivalence on the oracle step (golden weights, B = 3 -> shards)
        z = load_golden("spring_s12")
        cfg, B = O.cfg_from_golden(z)
        state = golden_weights(z)
        x = O.input_from_u8(z["input_u8"])
        xs = x[:2] if rank == 0 else x[1:3]   # equal-size shards of a 4-seq global batch [0,1,1,2]
        _, _, g = O.train_step(state, cfg, xs)
        names = sorted(g)
        vec = torch.cat([g[k].reshape(-1).double() for k in names])
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)
        vec /= world
        if rank == 0:
            xg = torch.cat([x[:2], x[1:3]])
            _, _, gfull = O.train_step(state, cfg, xg)
            ref = torch.cat([gfull[k].reshape(-1).double() for k in names])
            err = float((vec - ref).abs().max() / ref.abs().max())
            assert err < 1e-5, err
        q.put((rank, "ok"))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_data_parallel_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, "ok"), (1, "ok")], res
