"""bench.py's rank launch: `bench.py --gpus N` runs N
ranks, either under a launcher (WORLD_SIZE set: it must equal N) or by
starting them itself.  The BASELINE metric is quoted "@ 1/2/4/8 MI355X";
the reference itself is single-device (runners/torch_run_physics.py:78).

CPU tests: the argument checks that refuse a run which would time the wrong
number of GPUs (no GPU is touched: the checks run before any HIP call).
GPU test: `--gpus 2` without a launcher, both ranks on cuda:0 over gloo
(PAIG_DIST_BACKEND=gloo, PAIG_BENCH_DEVICE=0: the one-GPU rehearsal of the
N-rank path; production is RCCL, one GPU per rank), whose line must report
2 GPUs, dp2 and the global batch of 2 x 100.
"""
import json
import math
import os
import subprocess
import sys

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
BENCH = os.path.join(REPO, "bench.py")


def _bench(args, env_extra, timeout):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "PAIG_BENCH_DEVICE",
              "PAIG_DIST_BACKEND"):
        env.pop(k, None)
    env.update(env_extra)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    return subprocess.run([sys.executable, "-u", BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_world_size_must_match_gpus():
    r = _bench(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0"}, 120)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=3" in r.stderr


def test_launcher_world_size_one_with_gpus_two_is_refused():
    r = _bench(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0"}, 120)
    assert r.returncode == 2 and "--gpus 2" in r.stderr


def test_more_gpus_than_visible_is_refused():
    r = _bench(["--gpus", "64"], {}, 120)
    assert r.returncode == 2 and "visible GPUs" in r.stderr


@pytest.mark.gpu
def test_bench_gpus2_runs_two_ranks():
    r = _bench(["--gpus", "2", "--steps", "3", "--warmup", "2", "--legs", "0", "--cpu_baseline", "0",
                "--probe_steps", "1", "--dataset", "4"],
               {"PAIG_DIST_BACKEND": "gloo", "PAIG_BENCH_DEVICE": "0", "OMP_NUM_THREADS": "2"}, 600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    d = json.loads(lines[0])
    print({k: d[k] for k in ("value", "n_gpus", "ms_per_step", "final_loss")})
    assert d["n_gpus"] == 2
    assert d["config"]["parallelism"] == "dp2"
    assert d["config"]["global_batch"] == 200
    assert d["config"]["split_graph"] is True
    assert math.isfinite(d["final_loss"]) and d["value"] > 0
