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

    python bench.py [--gpus N --steps K --warmup W]     (N > 1: starts N ranks itself)
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

--gpus must equal the launcher's WORLD_SIZE when one is set (else exit 2).

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
    ap.add_argument("--byte_targets", type=int, default=1,
                    help="decoders read their targets as the dataset's bytes; the gather converts only the "
                         "encoder's frames (DeviceDataIterator.bind_targets, bit-identical)")
    ap.add_argument("--conv_math", default="split", choices=["split", "fp32", "bf16"],
                    help="U-Net conv arithmetic: split = f16/bf16 hi+lo operands on the 16-bit matrix cores, "
                         "fp32-accurate (meets the 1e-4 parity bar; default); fp32 = f32-input MFMA; "
                         "bf16 = bf16 operands (config #2)")
    ap.add_argument("--legs", type=int, default=1, help="also time BASELINE configs #2-#5 (LEGS) in the same line")
    ap.add_argument("--leg_steps", type=int, default=10)
    ap.add_argument("--leg_warmup", type=int, default=3)
    ap.add_argument("--leg_render", type=int, default=64,
                    help="distinct synthetic sequences rendered per leg (tiled to the resident dataset)")
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
    # the reference's own code path is not on this box: its throughput
    # relative to the oracle's, measured once on the build container's CPU
    # (tools/time_reference.py, alternating steps), scales the oracle's value
    try:
        rows = json.load(open(os.path.join(PROFILES, "cpu_reference_vs_oracle.json")))["rows"]
        r = rows.get(f"seq{sl0}")
        if r:
            out["oracle_over_reference"] = r["oracle_over_reference"]
            out["reference_estimate"] = round(out["value"] / r["oracle_over_reference"], 3)
            out["reference_ratio_source"] = "profiles/cpu_reference_vs_oracle.json (tools/time_reference.py)"
    except (OSError, ValueError, KeyError):
        pass
    return out


# BASELINE.json configs #2-#5 (runners/torch_run_physics.py:49-75 presets),
# timed as extra legs of the same run, B per rank
LEGS = [
    ("config2_spring_bf16", "spring_color", 512, 50, "bf16"),
    ("config3_3bp", "3bp_color", 512, 20, "split"),
    ("config4_mnist", "mnist_spring_color", 256, 12, "split"),
    ("config5_bouncing_r96", "bouncing_balls", 1024, 100, "split"),
]
# task -> (cell, input_steps, pred_steps, frame size): runners/torch_run_physics.py:49-75
TASKS = {"spring_color": ("spring_ode_cell", 4, 6, 32), "spring_color_half": ("spring_ode_cell", 4, 6, 32),
         "bouncing_balls": ("bouncing_ode_cell", 4, 6, 32), "3bp_color": ("gravity_ode_cell", 4, 12, 36),
         "mnist_spring_color": ("spring_ode_cell", 3, 7, 64)}


def run_workload(a, world, rank, dev, task, batch, seq_len, conv_math, steps, warmup, probe_steps, n_render):
    """One timed training workload: returns seqs/s over all ranks, the step
    time, the final loss, the per-kernel probe summaries and the dataset."""
    from paig_reproduction_amd.nn.datasets.synth import render_sequences
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet
    from paig_reproduction_amd.nn.datasets.iterators import DeviceDataIterator
    from paig_reproduction_amd import engine as E
    from paig_reproduction_amd.graph_step import GraphStep

    cell, ins, pred, size = TASKS[task]
    torch.manual_seed(0)
    m = PhysicsNet(task, 100, 1, cell, seq_len, ins, pred, a.ae, False, True, size * size,
                   "conv_encoder", "conv_st_decoder", device=dev).to(dev)
    m.conv_math = conv_math
    m.build_optimizer(a.lr, "rmsprop", True)
    if world > 1:
        for t in m.state_dict().values():
            dist.broadcast(t, 0)

    # resident synthetic dataset (this rank's shard): n_render rendered
    # sequences tiled to a.dataset batches; every step gathers the next B of a
    # shuffled epoch into the graph's fixed input buffer (get_batch)
    u8 = render_sequences(task, n_render, seq_len, seed=1000 * rank + 1)
    reps = max(1, -(-a.dataset * batch // n_render)) if n_render < 2 * batch else max(1, a.dataset // 2)
    u8 = np.concatenate([u8] * reps, 0)
    it = DeviceDataIterator(u8, (seq_len, 3, size, size), dev, seed=rank)
    xbuf = torch.empty((batch, seq_len, 3, size, size), device=dev)

    gstep = GraphStep(m, xbuf, world, split=None if a.split_graph < 0 else bool(a.split_graph), graph=bool(a.graph),
                      optimizer_in_graph=bool(a.graph_optimizer))
    eng = gstep.eng
    if a.byte_targets:
        eng.byte_targets = it.bind_targets(xbuf, ins + pred)

    def eager_step():
        it.next_batch(batch, out=xbuf)
        return gstep.eager()

    for i in range(warmup):
        eager_step()
    gstep.capture()

    def step():
        it.next_batch(batch, out=xbuf)   # get_batch: one gather launch, no H2D
        return gstep()

    step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # an event after every step (stream-ordered, no sync): per-step device
    # intervals for the median; `value` stays the whole-loop mean
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(steps):
        loss = step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    gstep.finish()
    per = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    med_ms = per[len(per) // 2] if len(per) % 2 else 0.5 * (per[len(per) // 2 - 1] + per[len(per) // 2])
    lossv = float(loss.item())
    # roofline probes: every tagged main-stream launch timed with HIP events
    # on its stream, over eager steps of the same workload after the timed region
    probe = E.KernelProbe(None)
    eng.probe = probe
    for i in range(probe_steps):
        eager_step()
    eng.probe = None
    kds = probe.summaries()
    res = {"value": world * batch * steps / el, "el": el, "med_ms": med_ms, "loss": lossv, "kds": kds, "split": gstep.split,
           "opt_in_graph": gstep.opt_in_graph, "byte_targets": eng.byte_targets is not None, "dataset_seqs": int(u8.shape[0]), "ins": ins, "pred": pred, "size": size,
           "u8_head": u8[:100]}
    del gstep, m, eng, it, xbuf
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


PEAK_F16_TFLOPS = 2500.0   # dense 16-bit MFMA (f16 / bf16), MI355X_MICROARCH.md
MFMA_FAMILIES = ("conv_fwd", "conv_dgrad", "conv_wgrad", "conv_bwd", "gemm_fwd", "gemm_wgrad", "gemm_dgrad")


def mfma_roof(conv_math):
    """(matrix-core FLOPs issued per algorithmic FLOP, peak TFLOP/s) of the
    MFMA kernels: split = 3 f16 MFMAs per product (hi*hi + hi*lo + lo*hi),
    bf16 = 1, fp32 = the f32-input MFMA at the fp32 rate."""
    return {"split": (3, PEAK_F16_TFLOPS), "bf16": (1, PEAK_F16_TFLOPS), "fp32": (1, PEAK_FP32_TFLOPS)}[conv_math]


def roof_of(kd, conv_math):
    """Both roofs of one probed launch: HBM (algorithmic bytes / launch time
    vs 8 TB/s) and, for the matrix-core kernels, MFMA (the FLOPs the matrix
    cores issue / launch time vs their dense peak); `bound` / `frac` are the
    binding one (the larger fraction)."""
    sec = kd["avg_ms"] * 1e-3
    tflops = kd["flops"] / sec / 1e12
    gbs = kd["bytes"] / sec / 1e9
    fam = kd["tag"].split(":")[0]
    hbm_frac = gbs / PEAK_HBM_GBS
    mfma = None
    if fam in MFMA_FAMILIES and kd["flops"]:
        mult, peak = mfma_roof(conv_math)
        mfma = {"achieved": round(mult * tflops, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(mult * tflops / peak, 4), "mfma_flops_per_flop": mult}
    out = {"kernel": kd["tag"], "avg_us": round(kd["avg_ms"] * 1e3, 2),
           "avg_us_events_raw": round(kd["avg_ms_raw"] * 1e3, 2), "event_overhead_us": round(kd["overhead_ms"] * 1e3, 2),
           "launches": kd["n"], "algorithmic_flops": kd["flops"], "algorithmic_bytes": kd["bytes"],
           "algorithmic_tflops": round(tflops, 2),
           "hbm": {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(hbm_frac, 4)},
           "mfma": mfma}
    if mfma is not None and mfma["frac"] > hbm_frac:
        out.update({"bound": "mfma", "achieved": mfma["achieved"], "peak": mfma["peak"], "unit": "TFLOP/s",
                    "frac": mfma["frac"]})
    else:
        out.update({"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(hbm_frac, 4)})
    return out


# the fixed headline probe, comparable across rounds: the backward of the
# ShallowUNet's c11 (24 -> 8 channels at 32 x 32; wgrad + dgrad, or the fused
# backward kernel when the layer runs one)
HEADLINE_LAYER = "c11"


def headline_roof(kds, conv_math):
    parts = [t for t in ("conv_bwd:" + HEADLINE_LAYER, "conv_wgrad:" + HEADLINE_LAYER,
                         "conv_dgrad:" + HEADLINE_LAYER) if t in kds]
    if not parts:
        return None
    agg = {"tag": "conv_bwd:" + HEADLINE_LAYER, "n": min(kds[t]["n"] for t in parts),
           "avg_ms": sum(kds[t]["avg_ms"] for t in parts), "avg_ms_raw": sum(kds[t]["avg_ms_raw"] for t in parts),
           "overhead_ms": kds[parts[0]]["overhead_ms"],
           "flops": sum(kds[t]["flops"] for t in parts), "bytes": sum(kds[t]["bytes"] for t in parts)}
    r = roof_of(agg, conv_math)
    r["launch_tags"] = parts
    return r


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """`--gpus N` (N > 1) without a launcher: start N fresh child processes,
    one rank per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on
    127.0.0.1), as `torch.distributed.run --nproc-per-node N` would, and exit
    with the first failing rank's status.  This process never touches the GPU
    (no HIP call before the children start; device_count() does not initialise
    it).  Rank 0 inherits stdout and prints the one JSON line; a rank that
    fails takes the others down with it (a rank left waiting in a collective
    would otherwise hang)."""
    import signal
    import subprocess
    if not os.environ.get("PAIG_BENCH_DEVICE") and torch.cuda.device_count() < n:
        print(f"bench.py: --gpus {n} but {torch.cuda.device_count()} visible GPUs", file=sys.stderr)
        sys.exit(2)
    base = dict(os.environ)
    base.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(free_port()), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    while procs:
        for p in list(procs):
            s = p.poll()
            if s is None:
                continue
            procs.remove(p)
            if s != 0 and rc == 0:
                rc = s if s > 0 else 128 - s
                for q in procs:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    sys.exit(rc)


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        launch_ranks(a.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world} (launch with --nproc-per-node {a.gpus}, "
              f"or without a launcher: bench.py starts the {a.gpus} ranks itself)", file=sys.stderr)
        sys.exit(2)
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

    r = run_workload(a, world, rank, dev, a.task, a.batch, a.seq_len, a.conv_math, a.steps, a.warmup, a.probe_steps,
                     2 * a.batch)
    el, kds = r["el"], r["kds"]
    ins, pred, size = r["ins"], r["pred"], r["size"]
    value = r["value"]
    top_kernel, top_src = summary_top()
    fam = tag_family(top_kernel)
    if a.probe != "auto":
        tag = a.probe
    else:
        cands = [t for t in kds if fam and t.startswith(fam)] or list(kds)
        tag = max(cands, key=lambda t: kds[t]["avg_ms"]) if cands else None

    roof = None
    traffic_path = a.traffic or default_traffic()
    traffic, step_bytes = pmc_traffic(traffic_path, tag, {"task": a.task, "batch": a.batch, "seq_len": a.seq_len,
                                                           "conv_math": a.conv_math})
    if tag in kds:
        roof = roof_of(kds[tag], a.conv_math)
        roof.update({"traffic": round(traffic) if traffic else None, "traffic_unit": "bytes/launch (PMC)",
                     "traffic_source": os.path.relpath(traffic_path, REPO) if traffic else None,
                     "summary_top_kernel": top_kernel, "summary": top_src})
    # the other large kernel families, for the record
    others = {}
    for want in ("dec_bwd:rollout", "dec_bwd:recon", "dec_fwd:rollout", "gemm_fwd:encoder.l1", "gemm_dgrad:encoder.l2",
                 "conv_wgrad:c11", "conv_fwd:c11", "conv_dgrad:c2", "conv_bwd:c11", "conv_bwd:c2"):
        if want in kds and want != tag:
            rr = roof_of(kds[want], a.conv_math)
            others[want] = {k: rr[k] for k in ("bound", "achieved", "unit", "frac", "avg_us")}
            others[want]["hbm_frac"] = rr["hbm"]["frac"]
            others[want]["mfma_frac"] = rr["mfma"]["frac"] if rr["mfma"] else None
    # BASELINE configs #2-#5 as extra legs (per-rank B, the same DP path)
    legs = {}
    if a.legs:
        for name, task, batch, seq_len, cm in LEGS:
            lr_ = run_workload(a, world, rank, dev, task, batch, seq_len, cm, a.leg_steps, a.leg_warmup,
                               a.probe_steps, min(2 * batch, a.leg_render))
            lk = lr_["kds"]
            # the leg's own top kernel: the probed main-stream launch family with the most time per step
            top = max(lk, key=lambda t: lk[t]["avg_ms"] * lk[t]["n"]) if lk else None
            ci, cp, cs = lr_["ins"], lr_["pred"], lr_["size"]
            legs[name] = {
                "metric": f"video-seqs/sec (train step) {task} B={batch}", "value": round(lr_["value"], 2),
                "unit": "video-seqs/s", "n_gpus": world, "steps": a.leg_steps, "warmup": a.leg_warmup,
                "ms_per_step": round(lr_["el"] / a.leg_steps * 1e3, 3), "dtype": "bf16" if cm == "bf16" else "fp32",
                "config": {"workload": f"{task} B={batch}/rank, {cs}x{cs}x3, seq_len {seq_len} ({ci} in / {cp} pred / "
                                       f"{seq_len - ci - cp} extrap)", "global_batch": world * batch,
                           "seq_len": seq_len, "parallelism": f"dp{world}", "conv_math": cm,
                           "dataset_seqs": lr_["dataset_seqs"]},
                "roofline": roof_of(lk[top], cm) if top else None, "final_loss": round(lr_["loss"], 4)}
    cpu = None
    if rank == 0 and world == 1 and a.cpu_baseline:
        cpu = cpu_baseline(a.task, r["u8_head"], a.ae, a.cpu_seconds, [a.seq_len] + ([12] if a.seq_len != 12 else []))
    if rank == 0:
        line = {
            "metric": METRIC if (a.task, a.batch) == ("spring_color", 100) else
            f"video-seqs/sec (train step) {a.task} B={a.batch}",
            "value": round(value, 2), "unit": "video-seqs/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 3), "ms_per_step_median": round(r["med_ms"], 4),
            "value_median": round(world * a.batch / (r["med_ms"] * 1e-3), 2),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16" if a.conv_math == "bf16" else "fp32",
            "data": "synthetic",
            "config": {"workload": f"{a.task} PhysicsNet train step (get_batch gather+fwd+loss+bwd+allreduce+RMSprop), "
                                   f"B={a.batch}/rank, {size}x{size}x3, seq_len {a.seq_len} "
                                   f"({ins} in / {pred} pred / {a.seq_len - ins - pred} extrap)",
                       "global_batch": world * a.batch, "seq_len": a.seq_len, "parallelism": f"dp{world}",
                       "conv_math": a.conv_math, "split_graph": r["split"],
                       "optimizer_in_graph": r["opt_in_graph"], "byte_targets": r["byte_targets"],
                       "dataset_seqs": r["dataset_seqs"]},
            "roofline": roof, "roofline_headline": headline_roof(kds, a.conv_math), "roofline_others": others, "cpu_baseline": cpu, "final_loss": round(r["loss"], 4),
            # whole-step memory-side traffic (committed PMC profile) at this run's step time
            "hbm_step": None if step_bytes is None else {
                "bytes_per_step": round(step_bytes), "achieved_GBs": round(step_bytes / (el / a.steps) / 1e9, 1),
                "peak_GBs": PEAK_HBM_GBS, "frac": round(step_bytes / (el / a.steps) / 1e9 / PEAK_HBM_GBS, 4)},
            "legs": legs,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def default_traffic():
    """The newest committed whole-step PMC traffic summary (profiles/rNN_pmc_traffic.json)."""
    import glob
    paths = sorted(glob.glob(os.path.join(PROFILES, "r*_pmc_traffic.json")))
    return paths[-1] if paths else os.path.join(PROFILES, "r02_pmc_traffic.json")


if __name__ == "__main__":
    main()
