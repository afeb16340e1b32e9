"""Benchmark: PhysicsNet training steps/s on MI355X (BASELINE.json metric
"video-seqs/sec (train step) spring_color B=100").

One step = batch fetch (the reference's get_batch, nn/network/base.py:57-63,
139-141: the next B sequences of a shuffled epoch, uint8/255 -> fp32 [B,T,C,H,W];
here one gather launch over a dataset resident in HBM), forward (encoder U-Net,
localiser, velocity MLP, 46-step physics rollout, STN decoder over all frames),
fused loss, backward, gradient all-reduce (N>1, RCCL), RMSprop — the
reference's train loop body (nn/network/base.py:139-152) in fresh-loss mode,
through the drop-in PhysicsNet API.  The dataset is synthetic spring_color
videos rendered on the host once (data="synthetic").

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
PROFILES = os.path.join(REPO, "profiles")


def summary_top(path=None):
    """Top kernel of the newest committed rocprof summary (profiles/rNN_summary_graph.txt)."""
    import glob
    import re
    paths = sorted(glob.glob(os.path.join(PROFILES, "r*_summary_graph.txt")))
    if path is None and not paths:
        return None, None
    path = path or paths[-1]
    for line in open(path):
        m = re.match(r"\s*[\d.]+%\s+([\d.]+)us/step n=\s*\d+ avg=\s*[\d.]+us (.*)$", line)
        if m:
            return m.group(2).strip(), os.path.relpath(path, REPO)
    return None, os.path.relpath(path, REPO)


def tag_family(kernel):
    """Engine probe-tag prefix of a kernel name (see engine.Engine._p sites)."""
    if kernel is None:
        return None
    if kernel.startswith("void "):
        kernel = kernel[5:]
    if kernel.startswith("dec_bwd"):
        return "dec_bwd:"
    if kernel.startswith("dec_fwd"):
        return "dec_fwd:"
    if kernel.startswith("conv_wgrad"):
        return "conv_wgrad:"
    if kernel.startswith("conv_fwd"):
        # template <CIN, COUT, H, W, KS, DG, UPS, PM>
        args = kernel[kernel.index("<") + 1:kernel.rindex(">")].split(",")
        return "conv_dgrad:" if args[5].strip() == "true" else "conv_fwd:"
    if kernel.startswith("gemm_split_k") or kernel.startswith("gemm_k"):
        ta, tb = [a.strip() for a in kernel[kernel.index("<") + 1:].split(",")[:2]]
        return {("false", "true"): "gemm_fwd:", ("true", "false"): "gemm_wgrad:",
                ("false", "false"): "gemm_dgrad:"}.get((ta, tb))
    return None


def pmc_traffic(path, tag, cfg):
    """(bytes per launch of the probed kernel, memory-side bytes per step) from
    the committed PMC summary of the same workload, or (None, None)."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    if {k: d.get("config", {}).get(k) for k in cfg} != cfg:
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
    ap.add_argument("--dataset", type=int, default=8, help="resident dataset size in batches (one epoch)")
    ap.add_argument("--probe", default="auto", help="kernel tag of the roofline object (auto: the longest "
                    "launch of the family of the top kernel in the newest committed profiles/rNN_summary_graph.txt)")
    ap.add_argument("--traffic", default=None,
                    help="committed rocprofv3 FETCH_SIZE/WRITE_SIZE summary (tools/pmc_traffic.py)")
    ap.add_argument("--graph", type=int, default=1, help="capture fwd+loss+bwd in a HIP graph (the batch "
                    "gather is launched eagerly before each replay)")
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
    ap.add_argument("--cpu_seconds", type=float, default=10.0, help="CPU time budget per cpu_baseline sample")
    return ap.parse_args()


def host_cores():
    """(threads to use, description): the CPUs this process may run on,
    capped by a cgroup CPU quota when one is set (a shared box)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    n = min(aff, quota) if quota else aff
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, f"{model}; affinity {aff} CPUs" + (f", cgroup quota {quota} CPUs" if quota else "")


def cpu_baseline(task, u8, ae, budget_s, seq_lens):
    """The oracle (torch CPU restatement of the reference, pinned to the
    reference's golden vectors) timed on the reference's workload: fresh-mode
    train steps of B sequences (config #1: B=100) at each seq_len, on this
    host's cores; a bounded number of steps (budget_s each)."""
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from oracle import physics_oracle as O
    from paig_reproduction_amd.nn.datasets.synth import as_model_input
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet

    threads, cores_desc = host_cores()
    torch.set_num_threads(threads)
    cell, _, _, ins, pred, size, _ = O.TASKS[task]
    res = {}
    for sl in seq_lens:
        cfg = O.Cfg(task, cell, sl, ins, pred, size, ae)
        torch.manual_seed(0)
        m = PhysicsNet(task, 100, 1, cell, sl, ins, pred, ae, False, True, size * size, "", "conv_st_decoder")
        state = {k: v.detach().clone() for k, v in m.state_dict().items()}
        x = torch.from_numpy(as_model_input(np.ascontiguousarray(u8[:, :sl])))
        O.train_step(state, cfg, x)  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            O.train_step(state, cfg, x)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget_s or n >= 50:
                break
        res[sl] = (x.shape[0] * n / el, n, el)
    sl0 = seq_lens[0]
    out = {"value": round(res[sl0][0], 3), "unit": "video-seqs/s", "cores": threads, "kind": "port",
           "sample": f"{res[sl0][1]} fresh-mode train steps x B={u8.shape[0]} ({task}, seq_len {sl0}) in "
                     f"{res[sl0][2]:.1f}s, oracle/physics_oracle.py on torch CPU, {threads} threads",
           "cpu": cores_desc}
    for sl in seq_lens[1:]:
        out[f"value_seq{sl}"] = round(res[sl][0], 3)
        out[f"sample_seq{sl}"] = f"{res[sl][1]} steps x B={u8.shape[0]} at seq_len {sl} in {res[sl][2]:.1f}s"
    return out


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

    # resident synthetic dataset (this rank's shard): 2B rendered sequences
    # tiled to a.dataset batches; every step gathers the next B of a
    # shuffled epoch into the graph's fixed input buffer (get_batch)
    from paig_reproduction_amd.nn.datasets.iterators import DeviceDataIterator
    u8 = render_sequences(a.task, 2 * a.batch, a.seq_len, seed=1000 * rank + 1)
    u8 = np.concatenate([u8] * max(1, a.dataset // 2), 0)
    it = DeviceDataIterator(u8, (a.seq_len, 3, size, size), dev, seed=rank)
    xbuf = torch.empty((a.batch, a.seq_len, 3, size, size), device=dev)

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

    def eager_step():
        it.next_batch(a.batch, out=xbuf)
        loss = body(xbuf)
        m.optimizer.step()
        return loss

    for i in range(a.warmup):
        eager_step()
    graph = None
    split = a.split_graph if a.split_graph >= 0 else int(world > 1)
    opt_in_graph = bool(a.graph and a.graph_optimizer and world == 1 and not split and m.optimizer.kind == "rmsprop")
    if a.graph:
        # fwd+loss+bwd (+RMSprop at N=1) captured once on the fixed input
        # buffer (two graphs when split); the gather, the DP all-reduce and
        # (N>1) the optimizer step stay eager
        torch.cuda.synchronize()
        if not split:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                lg = body(xbuf)
                if opt_in_graph:
                    m.optimizer.step()
            graph = ((g,), lg)
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
                    lg = body(xbuf)
                finally:
                    eng.bucket_hook = m._flat.allreduce_early
                g2.capture_end()
            torch.cuda.current_stream().wait_stream(cap)
            assert seen == [1], "backward did not reach the bucket split point"
            graph = ((g1, g2), lg)
        torch.cuda.synchronize()

    replays = [0]

    def step():
        if graph is None:
            return eager_step()
        gs, lg = graph
        it.next_batch(a.batch, out=xbuf)   # get_batch: one gather launch, no H2D
        replays[0] += 1
        gs[0].replay()
        if len(gs) == 2:
            m._flat.allreduce_early()   # overlaps the second graph (U-Net backward)
            gs[1].replay()
        if not opt_in_graph:
            m.optimizer.step()
        return lg

    step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if opt_in_graph:
        # the captured RMSprop step ran Python once, at capture: count its
        # replays (its lr is the captured constant; RMSprop only, see above)
        m.optimizer.steps += replays[0]
    lossv = float(loss.item())
    # roofline probes: every tagged main-stream launch timed with HIP events
    # on its stream, over eager steps of the same workload after the timed region
    probe = E.KernelProbe(None)
    eng.probe = probe
    for i in range(a.probe_steps):
        eager_step()
    eng.probe = None
    kds = probe.summaries()

    seqs = world * a.batch * a.steps
    value = seqs / el
    top_kernel, top_src = summary_top()
    fam = tag_family(top_kernel)
    if a.probe != "auto":
        tag = a.probe
    else:
        cands = [t for t in kds if fam and t.startswith(fam)] or list(kds)
        tag = max(cands, key=lambda t: kds[t]["avg_ms"]) if cands else None

    def roof_of(kd):
        sec = kd["avg_ms"] * 1e-3
        tflops = kd["flops"] / sec / 1e12
        if a.conv_math == "fp32" and kd["tag"].split(":")[0] in ("conv_fwd", "conv_dgrad", "conv_wgrad", "gemm_fwd",
                                                               "gemm_wgrad", "gemm_dgrad"):
            # f32-input MFMA: bounded by the fp32 matrix rate
            return {"bound": "mfma", "kernel": kd["tag"], "achieved": round(tflops, 3), "peak": PEAK_FP32_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(tflops / PEAK_FP32_TFLOPS, 4), "avg_us": round(kd["avg_ms"] * 1e3, 2),
                    "launches": kd["n"], "algorithmic_flops": kd["flops"], "algorithmic_bytes": kd["bytes"]}
        # 16-bit matrix cores / VALU kernels: HBM-bound; achieved = algorithmic
        # bytes per launch / launch time
        gbs = kd["bytes"] / sec / 1e9
        return {"bound": "hbm", "kernel": kd["tag"], "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_tflops": round(tflops, 2),
                "avg_us": round(kd["avg_ms"] * 1e3, 2), "avg_us_events_raw": round(kd["avg_ms_raw"] * 1e3, 2),
                "event_overhead_us": round(kd["overhead_ms"] * 1e3, 2), "launches": kd["n"],
                "algorithmic_flops": kd["flops"],
                "algorithmic_bytes": kd["bytes"]}

    roof = None
    traffic_path = a.traffic or os.path.join(PROFILES, "r02_pmc_traffic.json")
    traffic, step_bytes = pmc_traffic(traffic_path, tag, {"task": a.task, "batch": a.batch, "seq_len": a.seq_len,
                                                           "conv_math": a.conv_math})
    if tag in kds:
        roof = roof_of(kds[tag])
        roof.update({"traffic": round(traffic) if traffic else None, "traffic_unit": "bytes/launch (PMC)",
                     "summary_top_kernel": top_kernel, "summary": top_src})
    # the other large kernel families, for the record
    others = {}
    for want in ("dec_bwd:rollout", "dec_fwd:rollout", "gemm_fwd:encoder.l1", "gemm_dgrad:encoder.l2",
                 "conv_wgrad:c11", "conv_fwd:c11", "conv_dgrad:c2"):
        if want in kds and want != tag:
            r = roof_of(kds[want])
            others[want] = {k: r[k] for k in ("bound", "achieved", "unit", "frac", "avg_us")}
    cpu = None
    if rank == 0 and world == 1 and a.cpu_baseline:
        cpu = cpu_baseline(a.task, u8[:100], a.ae, a.cpu_seconds, [a.seq_len] + ([12] if a.seq_len != 12 else []))
    if rank == 0:
        line = {
            "metric": METRIC if (a.task, a.batch) == ("spring_color", 100) else
            f"video-seqs/sec (train step) {a.task} B={a.batch}",
            "value": round(value, 2), "unit": "video-seqs/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16" if a.conv_math == "bf16" else "fp32",
            "data": "synthetic",
            "config": {"workload": f"{a.task} PhysicsNet train step (get_batch gather+fwd+loss+bwd+allreduce+RMSprop), "
                                   f"B={a.batch}/rank, {size}x{size}x3, seq_len {a.seq_len} "
                                   f"({ins} in / {pred} pred / {a.seq_len - ins - pred} extrap)",
                       "global_batch": world * a.batch, "seq_len": a.seq_len, "parallelism": f"dp{world}",
                       "conv_math": a.conv_math, "split_graph": bool(a.graph and split),
                       "optimizer_in_graph": opt_in_graph, "dataset_seqs": int(u8.shape[0])},
            "roofline": roof, "roofline_others": others, "cpu_baseline": cpu, "final_loss": round(lossv, 4),
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
