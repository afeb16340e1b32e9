"""Shared test helpers: golden fixture loading and the parity comparison."""
import glob
import os

import numpy as np
import torch

from weights import golden_state

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GOLDEN = sorted(os.path.basename(p)[len("golden_"):-len(".npz")]
                for p in glob.glob(os.path.join(GOLDEN_DIR, "golden_*.npz")))

# Parity bar (north star): 1e-4 relative in fp32, measured normwise:
#   max|a - b| <= RTOL * max|b|  (elementwise-relative fails on exact zeros).
RTOL = 1e-4


def load_golden(name):
    return np.load(os.path.join(GOLDEN_DIR, f"golden_{name}.npz"), allow_pickle=False)


def golden_weights(z, seed=0):
    shapes = {}
    for s in z["state_shapes"]:
        k, shp, dt = str(s).split("|")
        shapes[k] = (tuple(int(d) for d in shp.split(",")) if shp else (), dt)
    return {k: torch.from_numpy(np.array(v, copy=True)) for k, v in golden_state(shapes, seed).items()}


def rel_err(a, b):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, dtype=np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    scale = max(np.abs(b).max(), 1e-30) if b.size else 1.0
    return float(np.abs(a - b).max() / scale) if b.size else 0.0


def assert_close(a, b, rtol=RTOL, what=""):
    e = rel_err(a, b)
    assert e <= rtol, f"{what}: normwise rel err {e:.3e} > {rtol:.1e}"
    return e


def grad_checks(z, grads, rtol, prefix=""):
    """Compare a {key: grad tensor} dict with the fixture's full grads / summaries."""
    errs = {}
    for k in [str(s) for s in z["grad_keys"]]:
        assert k in grads, f"{prefix}missing grad {k}"
        g = grads[k].detach().cpu().double().numpy()
        if "grad/" + k in z.files:
            errs[k] = assert_close(g, z["grad/" + k], rtol, f"{prefix}grad {k}")
        else:
            g2 = g.reshape(g.shape[0], -1)
            errs[k + "[sum0]"] = assert_close(g2.sum(0), z["gradsum0/" + k], rtol, f"{prefix}gradsum0 {k}")
            errs[k + "[sum1]"] = assert_close(g2.sum(1), z["gradsum1/" + k], rtol, f"{prefix}gradsum1 {k}")
            errs[k + "[slice]"] = assert_close(g2[:64, :64], z["gradslice/" + k], rtol, f"{prefix}gradslice {k}")
            n = np.linalg.norm(g2)
            assert abs(n - float(z["gradnorm/" + k])) <= rtol * float(z["gradnorm/" + k]) + 1e-30, k
    return errs
