"""Deterministic, order-independent parameter generator shared by the golden
fixture generator (``gen_golden.py``) and the tests.

Fixtures store outputs, not the ~9 MB of weights: both sides regenerate the
same state_dict from ``(key, shape, seed)`` alone.
"""
import zlib

import numpy as np

# 0-dim float64 physics parameters (nn/network/cells.py:28-29,92-93) and the
# frozen float32 dt: fixed, non-trivial values so the exp() paths are exercised.
SCALARS = {
    "rollout_cell.k": 0.11,
    "rollout_cell.equil": -0.07,
    "rollout_cell.g": 0.05,
    "rollout_cell.m": 0.0,
}


def golden_state(shapes, seed=0):
    """shapes: dict key -> (tuple shape, numpy dtype str). Returns dict of numpy arrays."""
    out = {}
    fan = {}
    for key, (shape, _) in shapes.items():
        if key.endswith("weight") and len(shape) >= 2:
            fan[key[: -len("weight")]] = int(np.prod(shape[1:]))
    for key, (shape, dt) in shapes.items():
        if key in SCALARS:
            out[key] = np.array(SCALARS[key], dtype=dt)
            continue
        if key.endswith(".dt"):
            out[key] = np.array({"rollout_cell.dt": 0.3}.get(key, 0.3), dtype=dt)
            continue
        rng = np.random.default_rng((zlib.crc32(key.encode()) ^ (seed * 7919)) & 0xFFFFFFFF)
        unet = key.startswith("encoder.shallow_unet.") or key.startswith("encoder.unet.")
        if unet and key.endswith("bias"):
            # keep the ReLU U-Net alive (with torch-default scales its ReLU'd
            # output is identically 0 and every U-Net gradient vanishes)
            out[key] = rng.uniform(-0.1, 0.2, size=shape).astype(dt)
            continue
        if key.startswith("encoder.l3.") and key.endswith("bias"):
            out[key] = rng.uniform(-1.0, 1.0, size=shape).astype(dt)  # spread positions over the frame
            continue
        if key.endswith("weight") and len(shape) >= 2:
            b = 1.0 / np.sqrt(fan[key[: -len("weight")]])
            if unet:
                b *= np.sqrt(6.0)            # He-uniform gain
            if key.startswith("encoder.l3."):
                b *= 4.0
        elif key.endswith("bias"):
            prefix = key[: -len("bias")]
            b = 1.0 / np.sqrt(fan.get(prefix, shape[0] if len(shape) else 1))
        elif key.endswith("bias_ih") or key.endswith("bias_hh") or "weight_" in key:
            b = 0.5
        else:
            b = 0.1
        out[key] = rng.uniform(-b, b, size=shape).astype(dt)
    return out
