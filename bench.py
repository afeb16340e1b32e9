"""Benchmark: PhysicsNet training steps/s on MI355X (BASELINE.json metric
"video-seqs/sec (train step) spring_color B=100").

One step = forward (encoder U-Net, localiser, velocity MLP, 46-step physics
rollout, STN decoder over all frames), fused loss, backward, gradient
all-reduce (N>1, RCCL), RMSprop — the reference's train loop body
(nn/network/base.py:139-152) in fresh-loss mode, through the drop-in
PhysicsNet API.  Inputs are synthetic spring_color videos rendered on the host
once and kept resident in HBM (data="synthetic").

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Weak scaling: B sequences per rank.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 (vector == f32 MFMA), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
METRIC = "video-seqs/sec (train step) spring_color B=100 @ 1/2/4/8 MI355X"   # BASELINE.json
DOMINANT = "conv_wgrad:c11"   # largest kernel in profiles/r01_summary_eager.txt


def pmc_traffic(path, tag, cfg):
    """(bytes per launch of the probed kernel, memory-side bytes per step) from
    the committed PMC summary of the same workload, or (None, None)."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    if d.get("config") != cfg:
        return None, None
    kern = d.get("probe_kernels", {}).get(tag)
    per = d["kernels"].get(kern, {}).get("traffic_bytes") if kern else None
    step = sum(v["traffic_bytes"] * v["launches"] for v in d["kernels"].values()) / d.get("steps_profiled", 1)
    return per, step


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=100, help="sequences per rank")
    ap.add_argument("--task", default="spring_color")
    ap.add_argument("--seq_len", type=int, default=50, help="4 in / 6 pred / 40 extrap")
    ap.add_argument("--ae", type=float, default=3.0)
    ap.add_argument("--lr", type=float, default=6e-4)
    ap.add_argument("--nbatches", type=int, default=4, help="distinct resident batches cycled through")
    ap.add_argument("--probe", default="auto", help="kernel tag timed with HIP events for the roofline "
                    "(auto: the dominant kernel of the committed rocprof profile)")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "r01_pmc_traffic.json"),
                    help="committed rocprofv3 FETCH_SIZE/WRITE_SIZE summary (tools/pmc_traffic.py)")
    ap.add_argument("--graph", type=int, default=1, help="capture fwd+loss+bwd in a HIP graph per resident batch")
    ap.add_argument("--probe_steps", type=int, default=5, help="eager steps timing the probed kernel")
    ap.add_argument("--graph_optimizer", type=int, default=1,
                    help="at N=1 capture the RMSprop launch in the step graph too (it runs every replay; "
                         "no all-reduce to order it after, no step counter in RMSprop)")
    ap.add_argument("--split_graph", type=int, default=-1,
                    help="capture the step as two HIP graphs split where the early gradient bucket is final, and "
                         "all-reduce that bucket between the replays, overlapping the U-Net backward "
                         "(-1: on when N > 1)")
    ap.add_argument("--conv_math", default="split", choices=["split", "fp32", "bf16"],
                    help="U-Net conv arithmetic: split = f16/bf16 hi+lo operands on the 16-bit matrix cores, "
                         "fp32-accurate (meets the 1e-4 parity bar; default); fp32 = f32-input MFMA; "
                         "bf16 = bf16 operands (config #2)")
    ap.add_argument("--cpu_baseline", type=int, default=1)
    ap.add_argument("--cpu_seconds", type=float, default=15.0)
    return ap.parse_args()


def cpu_baseline(task, seq_len, ae, budget_s):
    """The oracle (torch CPU restatement of the reference, pinned to the
    reference's golden vectors) timed on a bounded sample of the same
    workload: fresh-mode train steps of B_s sequences at the same seq_len."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from oracle import physics_oracle as O
    from paig_reproduction_amd.nn.datasets.synth import render_sequences, as_model_input
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cell, _, _, ins, pred, size, _ = O.TASKS[task]
    cfg = O.Cfg(task, cell, seq_len, ins, pred, size, ae)
    torch.manual_seed(0)
    m = PhysicsNet(task, 100, 1, cell, seq_len, ins, pred, ae, False, True, size * size, "", "conv_st_decoder")
    state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    Bs = 10
    x = torch.from_numpy(as_model_input(render_sequences(task, Bs, seq_len, seed=7)))
    O.train_step(state, cfg, x)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        O.train_step(state, cfg, x)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 50:
            break
    return {"value": round(n * Bs / el, 3), "unit": "video-seqs/s", "cores": threads, "kind": "port",
            "sample": f"{n} fresh-mode train steps x {Bs} seqs ({task}, seq_len {seq_len}), oracle/physics_oracle.py "
                      f"on torch CPU, {threads} threads, {el:.1f}s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PAIG_DIST_BACKEND=gloo / PAIG_BENCH_DEVICE=0 rehearse the N-rank code path
    # with several ranks on ONE GPU (the production path is RCCL, one GPU per rank)
    backend = os.environ.get("PAIG_DIST_BACKEND", "nccl")
    local = int(os.environ.get("PAIG_BENCH_DEVICE", local))
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local}")

    from paig_reproduction_amd.nn.datasets.synth import render_sequences, as_model_input
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet
    from paig_reproduction_amd import engine as E

    # task -> (cell, input_steps, pred_steps, frame size): runners/torch_run_physics.py:49-75
    tasks = {"spring_color": ("spring_ode_cell", 4, 6, 32), "spring_color_half": ("spring_ode_cell", 4, 6, 32),
             "bouncing_balls": ("bouncing_ode_cell", 4, 6, 32), "3bp_color": ("gravity_ode_cell", 4, 12, 36),
             "mnist_spring_color": ("spring_ode_cell", 3, 7, 64)}
    cell, ins, pred, size = tasks[a.task]
    torch.manual_seed(0)
    m = PhysicsNet(a.task, 100, 1, cell, a.seq_len, ins, pred, a.ae, False, True, size * size,
                   "conv_encoder", "conv_st_decoder", device=dev).to(dev)
    m.conv_math = a.conv_math
    m.build_optimizer(a.lr, "rmsprop", True)
    if world > 1:
        for t in m.state_dict().values():
            dist.broadcast(t, 0)

    data = [torch.from_numpy(as_model_input(render_sequences(a.task, a.batch, a.seq_len, seed=1000 * rank + i)))
            .to(dev) for i in range(a.nbatches)]

    probe = E.KernelProbe(a.probe if a.probe != "auto" else DOMINANT)
    eng = m._native()

    seed_grad = {}

    def body(x):
        m.output = m(x)
        loss, _ = m.compute_loss()
        m.optimizer.zero_grad(set_to_none=True)
        # d loss / d loss = 1 from a persistent tensor (made before any graph
        # capture): autograd's implicit ones_like would be a fill kernel per step
        if "one" not in seed_grad:
            seed_grad["one"] = torch.ones_like(loss)
        loss.backward(seed_grad["one"])
        return loss

    def eager_step(i):
        loss = body(data[i % len(data)])
        m.optimizer.step()
        return loss

    for i in range(a.warmup):
        eager_step(i)
    graphs = None
    split = a.split_graph if a.split_graph >= 0 else int(world > 1)
    opt_in_graph = bool(a.graph and a.graph_optimizer and world == 1 and not split and m.optimizer.kind == "rmsprop")
    if a.graph:
        # one graph per resident batch (two when split), sharing one memory
        # pool; the optimizer step and the DP all-reduce stay eager
        torch.cuda.synchronize()
        graphs, pool = [], None
        for x in data:
            if not split:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    lg = body(x)
                    if opt_in_graph:
                        m.optimizer.step()
                pool = g.pool()
                graphs.append(((g,), lg))
                continue
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
                g1.capture_begin(pool=pool, capture_error_mode="relaxed")
                eng.bucket_hook = cut
                try:
                    lg = body(x)
                finally:
                    eng.bucket_hook = m._flat.allreduce_early
                g2.capture_end()
            torch.cuda.current_stream().wait_stream(cap)
            assert seen == [1], "backward did not reach the bucket split point"
            pool = g1.pool()
            graphs.append(((g1, g2), lg))
        torch.cuda.synchronize()

    def step(i):
        if graphs is None:
            return eager_step(i)
        gs, lg = graphs[i % len(graphs)]
        gs[0].replay()
        if len(gs) == 2:
            m._flat.allreduce_early()   # overlaps the second graph (U-Net backward)
            gs[1].replay()
        if not opt_in_graph:
            m.optimizer.step()
        return lg

    step(0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    lossv = float(loss.item())
    # roofline probe: the dominant kernel timed with HIP events on its stream,
    # over eager steps of the same workload right after the timed region
    eng.probe = probe
    for i in range(a.probe_steps):
        eager_step(i)
    eng.probe = None

    seqs = world * a.batch * a.steps
    value = seqs / el
    kd = probe.summary()
    roof = None
    traffic, step_bytes = pmc_traffic(a.traffic, probe.tag, {"task": a.task, "batch": a.batch, "seq_len": a.seq_len})
    if kd is not None:
        sec = kd["avg_ms"] * 1e-3
        tflops = kd["flops"] / sec / 1e12
        if a.conv_math == "fp32":
            # f32-input MFMA: bounded by the fp32 matrix rate
            roof = {"bound": "mfma", "kernel": kd["tag"], "achieved": round(tflops, 3), "peak": PEAK_FP32_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(tflops / PEAK_FP32_TFLOPS, 4)}
        else:
            # 16-bit matrix cores: the kernel's arithmetic is ~1/5 of the f32 form,
            # so HBM bounds it; achieved = algorithmic bytes / launch time
            gbs = kd["bytes"] / sec / 1e9
            roof = {"bound": "hbm", "kernel": kd["tag"], "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_tflops": round(tflops, 2)}
        roof.update({"traffic": round(traffic) if traffic else None, "traffic_unit": "bytes/launch (PMC)",
                     "avg_us": round(kd["avg_ms"] * 1e3, 2), "launches": kd["n"], "algorithmic_flops": kd["flops"],
                     "algorithmic_bytes": kd["bytes"]})
    cpu = None
    if rank == 0 and world == 1 and a.cpu_baseline:
        cpu = cpu_baseline(a.task, a.seq_len, a.ae, a.cpu_seconds)
    if rank == 0:
        line = {
            "metric": METRIC if (a.task, a.batch) == ("spring_color", 100) else
            f"video-seqs/sec (train step) {a.task} B={a.batch}",
            "value": round(value, 2), "unit": "video-seqs/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16" if a.conv_math == "bf16" else "fp32",
            "data": "synthetic",
            "config": {"workload": f"{a.task} PhysicsNet train step (fwd+loss+bwd+allreduce+RMSprop), "
                                   f"B={a.batch}/rank, {size}x{size}x3, seq_len {a.seq_len} "
                                   f"({ins} in / {pred} pred / {a.seq_len - ins - pred} extrap)",
                       "global_batch": world * a.batch, "seq_len": a.seq_len, "parallelism": f"dp{world}",
                       "conv_math": a.conv_math, "split_graph": bool(a.graph and split),
                       "optimizer_in_graph": opt_in_graph},
            "roofline": roof, "cpu_baseline": cpu, "final_loss": round(lossv, 4),
            # whole-step memory-side traffic (committed PMC profile) at this run's step time
            "hbm_step": None if step_bytes is None else {
                "bytes_per_step": round(step_bytes), "achieved_GBs": round(step_bytes / (el / a.steps) / 1e9, 1),
                "peak_GBs": PEAK_HBM_GBS, "frac": round(step_bytes / (el / a.steps) / 1e9 / PEAK_HBM_GBS, 4)},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
