"""Synthetic video renderer.

The reference ships no data (its README points at an offline Google Drive
folder) and its generators need ``skimage.draw.circle`` plus TF dataset
downloads (``/root/reference/nn/datasets/generators.py:243-364,517-652``).
This module renders datasets of the same shape and file layout instead:
``npz`` with ``train_x / valid_x / test_x`` as ``uint8 [N, T, H, W, C]``
(NHWC, exactly what ``get_iterators`` expects, including quirk Q5 — the
loader reshapes instead of transposing).

Physics follows the generators' integrators (spring: ``generators.py:296-306``;
gravity and bouncing in the same spirit); disks are anti-aliased by 4x
supersampling, object ``j`` drawn on colour channel ``2-j``
(``generators.py:310-315``).
"""
import numpy as np

# task -> (n_objs, img_size, default seq_len, physics)
TASKS = {
    "spring_color": (2, 32, "spring"),
    "spring_color_half": (2, 32, "spring"),
    "bouncing_balls": (2, 32, "bounce"),
    "3bp_color": (3, 36, "gravity"),
    "mnist_spring_color": (2, 64, "spring"),
}


def _disk_frames(pos, radius, size, ss=4):
    """pos [T, K, 2] (x, y) in pixels -> float32 [T, K, size, size] coverage."""
    g = (np.arange(size * ss, dtype=np.float32) + 0.5) / ss
    T, K, _ = pos.shape
    dx = g[None, None, None, :] - pos[:, :, 0, None, None]
    dy = g[None, None, :, None] - pos[:, :, 1, None, None]
    inside = (dx * dx + dy * dy) <= radius * radius
    cov = inside.reshape(T, K, size, ss, size, ss).mean(axis=(3, 5))
    return cov.astype(np.float32)


def _spring_traj(rng, T, size, radius, k=4.0, equil=6.0, vmax=8.0, dt=0.3, sub=10, half=False):
    while True:
        lo, hi = radius + equil, size - (radius + equil)
        cm = lo + (hi - lo) * rng.random(2)
        if half:
            cm[0] = lo + (size / 2 - lo) * rng.random()
        ang = rng.random() * 2 * np.pi
        r = rng.random() + 0.5
        p = np.array([[np.cos(ang) * equil * r, np.sin(ang) * equil * r],
                      [-np.cos(ang) * equil * r, -np.sin(ang) * equil * r]]) + cm
        a = rng.random(2) * 2 * np.pi
        v = np.stack([np.cos(a) * vmax, np.sin(a) * vmax], axis=1) * rng.random((2, 1))
        out = np.zeros((T, 2, 2))
        ok = True
        for t in range(T):
            out[t] = p
            for _ in range(sub):
                d = p[0] - p[1]
                n = np.linalg.norm(d) + 1e-8
                F = k * (n - 2 * equil) * d / n
                v[0] -= dt / sub * F
                v[1] += dt / sub * F
                p = p + dt / sub * v
            if np.any(p < radius) or np.any(p > size - radius):
                ok = False
                break
        if ok:
            return out


def _bounce_traj(rng, T, size, radius, vmax=8.0, dt=0.3, sub=10):
    p = radius + (size - 2 * radius) * rng.random((2, 2))
    a = rng.random(2) * 2 * np.pi
    v = np.stack([np.cos(a), np.sin(a)], axis=1) * vmax * (0.5 + 0.5 * rng.random((2, 1)))
    out = np.zeros((T, 2, 2))
    for t in range(T):
        out[t] = p
        for _ in range(sub):
            p = p + dt / sub * v
            lo, hi = p < radius, p > size - radius
            v = np.where(lo | hi, -v, v)
            p = np.where(lo, 2 * radius - p, np.where(hi, 2 * (size - radius) - p, p))
    return out


def _gravity_traj(rng, T, size, radius, g=60.0, dt=0.5, sub=10):
    c = size / 2
    while True:
        ang = rng.random() * 2 * np.pi + np.array([0, 2 * np.pi / 3, 4 * np.pi / 3])
        r = 4 + 4 * rng.random()
        p = np.stack([c + r * np.cos(ang), c + r * np.sin(ang)], axis=1)
        sp = np.sqrt(g / r) * 0.35
        v = np.stack([-np.sin(ang), np.cos(ang)], axis=1) * sp
        out = np.zeros((T, 3, 2))
        for t in range(T):
            out[t] = p
            for _ in range(sub):
                acc = np.zeros_like(p)
                for i in range(3):
                    for j in range(3):
                        if i != j:
                            d = p[j] - p[i]
                            n = max(np.linalg.norm(d), 1.0)
                            acc[i] += g * d / n ** 3
                v = v + dt / sub * acc
                p = p + dt / sub * v
        if np.all(out > radius) and np.all(out < size - radius):
            return out


def render_sequences(task, n, seq_len, seed=0, radius=2.0):
    """Render ``n`` sequences -> uint8 [n, seq_len, H, W, 3] (NHWC)."""
    n_objs, size, phys = TASKS[task]
    rng = np.random.default_rng(seed)
    out = np.zeros((n, seq_len, size, size, 3), dtype=np.uint8)
    for i in range(n):
        if phys == "spring":
            scale = size / 32.0
            traj = _spring_traj(rng, seq_len, size, radius * scale, equil=6.0 * scale,
                                half=(task == "spring_color_half"))
            rad = radius * (3.0 if task == "mnist_spring_color" else 1.0)
        elif phys == "bounce":
            traj = _bounce_traj(rng, seq_len, size, radius)
            rad = radius
        else:
            traj = _gravity_traj(rng, seq_len, size, radius)
            rad = radius
        cov = _disk_frames(traj, rad, size)  # [T, K, H, W]
        frame = np.zeros((seq_len, size, size, 3), dtype=np.float32)
        if task == "mnist_spring_color":
            bg = np.clip(rng.random((size, size)).astype(np.float32) - 0.2, 0.0, 1.0)
            frame[:] = bg[None, :, :, None]
        for j in range(n_objs):
            ch = 2 - (j % 3)
            frame[..., ch] = np.maximum(frame[..., ch], cov[:, j])
        out[i] = (np.clip(frame, 0.0, 1.0) * 255).astype(np.uint8)
    return out


def write_dataset(path, task, seq_len, n_train, n_valid, n_test, seed=0):
    """Write an npz with the reference dataset layout (train_x/valid_x/test_x)."""
    tr = render_sequences(task, n_train, seq_len, seed)
    va = render_sequences(task, n_valid, seq_len, seed + 1)
    te = render_sequences(task, n_test, seq_len, seed + 2)
    np.savez_compressed(path, train_x=tr, valid_x=va, test_x=te)
    return path


def as_model_input(u8):
    """uint8 NHWC [N,T,H,W,C] -> float32 [N,T,C,H,W] with the reference's Q5
    reshape-not-transpose semantics (``nn/datasets/iterators.py:60-67``)."""
    N, T, H, W, C = u8.shape
    return (u8.astype(np.float32).reshape(N, T, C, H, W) / 255).astype(np.float32)
