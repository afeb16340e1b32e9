"""The HIP data-parallel training step on one GPU:
two fresh child processes (tests/workers/dp_step_worker.py) share cuda:0
over gloo and run 3 steps through bench.py's step (paig_reproduction_amd.
graph_step: the split HIP graph, allreduce_early between the replays,
FlatOptimizer.step with the late bucket and the fp64 scalars); a third child
runs the same steps single-process on the concatenated batches.  The
reference loop being replaced is single-process (nn/network/base.py:141-152);
the DP contract is that the averaged per-rank gradients of equal halves are
the full batch's gradient (the losses are batch means).

Every step is compared from the same starting state (the single-process
run loads the DP run's parameters and optimizer buffers before each step):
over several steps the two trajectories would part at the first near-tie
max-pool / ReLU decision that a one-ulp parameter difference flips, as any
two fp32 runs of the reference do.  Bars: 6e-6 normwise on every step's
all-reduced flat gradients (test_gpu_fullsize's halves bar, ~3x the
measured fp32 reassociation error) and, with momentum SGD (an update linear
in the gradient), on the updated parameters.  RMSprop's first update is
lr * sign(g) / sqrt(1 - alpha) for |g| >> eps, so a gradient component at
rounding-noise level can flip its parameter's update: for RMSprop the
updated parameters are reported, not bounded.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
WORKER = os.path.join(REPO, "tests", "workers", "dp_step_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, timeout=300):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = "2"
    return subprocess.Popen([sys.executable, "-u", WORKER] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                            env=env, text=True)


def _wait(procs, timeout=300):
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0 and "WORKER_OK" in out, out[-3000:]


def _rel(a, b):
    return float(np.abs(a.astype(np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("kind", ["momentum", "rmsprop"])
def test_dp_step_equals_single_process(kind, tmp_path):
    dp, single = tmp_path / "dp", tmp_path / "single"
    dp.mkdir()
    single.mkdir()
    port = _free_port()
    procs = [_run(["--mode", "dp", "--rank", str(r), "--world", "2", "--port", str(port), "--kind", kind,
                   "--out", str(dp)]) for r in range(2)]
    _wait(procs)
    _wait([_run(["--mode", "single", "--kind", kind, "--out", str(single), "--src", str(dp)])])
    for i in range(3):
        for nm in ("g32", "g64"):
            e = _rel(np.load(dp / f"post_{nm}_{i}.npy"), np.load(single / f"post_{nm}_{i}.npy"))
            assert e <= 6e-6, f"{kind} step {i}: all-reduced {nm} rel err {e:.3g}"
        ep = _rel(np.load(dp / f"post_p32_{i}.npy"), np.load(single / f"post_p32_{i}.npy"))
        e64 = _rel(np.load(dp / f"post_p64_{i}.npy"), np.load(single / f"post_p64_{i}.npy"))
        print(f"{kind} step {i}: updated parameters rel err fp32 {ep:.3g} fp64 {e64:.3g}")
        if kind == "momentum":
            assert ep <= 6e-6 and e64 <= 6e-6, (i, ep, e64)


@pytest.mark.parametrize("kind", ["rmsprop", "momentum"])
def test_rccl_world1_step_bit_identical(kind, tmp_path):
    """RCCL executed on the DP step's own path: a world-1
    `nccl` process group with FlatParams.FORCE_DP, so the split HIP graph
    runs, allreduce_early issues the asynchronous AVG of the early bucket on
    RCCL's stream between the two replays, and FlatOptimizer.step reduces the
    late bucket and the fp64 scalars and waits for the early work.  AVG over
    one rank is exact: every step's flat gradients and updated parameters must
    be bit-identical to the single-process step from the same state.  (No
    scaling claim: one GPU box holds one rank.)"""
    dp, single = tmp_path / "dp", tmp_path / "single"
    dp.mkdir()
    single.mkdir()
    _wait([_run(["--mode", "dp", "--rank", "0", "--world", "1", "--port", str(_free_port()), "--backend", "nccl",
                 "--force_dp", "--kind", kind, "--out", str(dp)])])
    _wait([_run(["--mode", "single", "--kind", kind, "--out", str(single), "--src", str(dp)])])
    for i in range(3):
        for nm in ("g32", "g64", "p32", "p64"):
            a, b = np.load(dp / f"post_{nm}_{i}.npy"), np.load(single / f"post_{nm}_{i}.npy")
            assert np.array_equal(a, b), f"{kind} step {i}: {nm} differs (max {np.abs(a - b).max():.3g})"
