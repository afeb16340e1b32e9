"""Dataset iterators (reference nn/datasets/iterators.py:4-69).

Same semantics: unseeded shuffle per epoch (an optional ``seed`` makes it
reproducible), drop-last (the epoch ends when ``start + batch > N``), uint8/255
to float32, and quirk Q5 — NHWC frames are RESHAPED (not transposed) to
[C, H, W].  ``--datapoints`` is a no-op exactly as in the reference (Q7).

Data-parallel: ``rank``/``world`` give each rank a disjoint slice of every
epoch's shared permutation (a shared ``seed`` keeps the permutations equal).

``DeviceDataIterator`` keeps the dataset in HBM as uint8 and
gathers each batch on the GPU (one HIP launch, /255 fused): same RNG draws,
same batches, no per-step host gather or H2D copy of frames.
"""
import numpy as np


class DataIterator:
    def __init__(self, X, Y=None, seed=None, rank=0, world=1):
        self.X = X
        self.Y = Y
        self.num_examples = self.X.shape[0]
        self.epochs_completed = 0
        self.indices = np.arange(self.num_examples)
        self.rng = np.random.default_rng(seed) if seed is not None else None
        self.rank, self.world = rank, world
        self.reset_iteration()

    def reset_iteration(self):
        if self.rng is not None:
            self.rng.shuffle(self.indices)
        else:
            np.random.shuffle(self.indices)
        self.start_idx = 0

    def get_epoch(self):
        return self.epochs_completed

    def reset_epoch(self):
        self.reset_iteration()
        self.epochs_completed = 0

    def _take(self, batch_size):
        """This rank's indices of the next global batch; drop-last epoch end."""
        gb = batch_size * self.world
        lo = self.start_idx + self.rank * batch_size
        idx = self.indices[lo:lo + batch_size].copy()
        self.start_idx += gb
        if self.start_idx + gb > self.num_examples:
            self.reset_iteration()
            self.epochs_completed += 1
        return idx

    def next_batch(self, batch_size, data_type="train", shuffle=True):
        assert data_type in ["train", "val", "test"], "data_type must be 'train', 'val', or 'test'."
        idx = self._take(batch_size)
        batch_x = self.X[idx]
        batch_y = self.Y[idx] if self.Y is not None else self.Y
        return (batch_x, batch_y)

    def sample_random_batch(self, batch_size):
        # reference quirk kept: the drawn start_idx is unused (iterators.py:42-47)
        np.random.randint(0, self.num_examples - batch_size)
        batch_x = self.X[self.start_idx:self.start_idx + batch_size]
        batch_y = self.Y[self.start_idx:self.start_idx + batch_size] if self.Y is not None else self.Y
        return (batch_x, batch_y)


class DeviceDataIterator(DataIterator):
    """DataIterator over a uint8 dataset resident on ``device``.

    ``X_u8``: uint8 [N, T, H, W, C] (the npz layout); ``shape``: the per-example
    model shape the bytes are reinterpreted as (Q5: (T, C, H, W)).
    next_batch returns a float32 device tensor [B, *shape] gathered by
    paig_gather_u8_f32; ``X`` is the device uint8 tensor (``X.shape[0]`` is N)."""

    def __init__(self, X_u8, shape, device, seed=None, rank=0, world=1):
        import torch
        self.shape = tuple(int(d) for d in shape)
        self.row = int(np.prod(X_u8.shape[1:]))
        assert self.row == int(np.prod(self.shape)), (X_u8.shape, shape)
        self.device = torch.device(device)
        super().__init__(torch.from_numpy(np.ascontiguousarray(X_u8)).to(self.device), None, seed, rank, world)

    def _gather(self, idx):
        import torch
        from paig_reproduction_amd._lib import lib, ptr, stream_handle
        idx = np.asarray(idx, dtype=np.int64)
        assert idx.size == 0 or (idx.min() >= 0 and idx.max() < self.num_examples)
        out = torch.empty((idx.size,) + self.shape, device=self.device)
        if idx.size:
            idx_d = torch.from_numpy(idx).pin_memory().to(self.device, non_blocking=True)
            lib().paig_gather_u8_f32(ptr(self.X), ptr(idx_d), ptr(out), int(idx.size), self.row,
                                     stream_handle(self.device))
        return out

    def next_batch(self, batch_size, data_type="train", shuffle=True):
        assert data_type in ["train", "val", "test"], "data_type must be 'train', 'val', or 'test'."
        return self._gather(self._take(batch_size)), None

    def sample_random_batch(self, batch_size):
        np.random.randint(0, self.num_examples - batch_size)   # reference quirk (iterators.py:42-47)
        return self._gather(np.arange(self.start_idx, min(self.start_idx + batch_size, self.num_examples))), None


def get_iterators(file, conv=False, datapoints=0, seed=None, rank=0, world=1, device=None):
    """``device``: keep the uint8 data on that GPU (DeviceDataIterator, F2)."""
    data = np.load(file)
    if conv:
        img_shape = data["train_x"][0, 0].shape
        img_shape = (img_shape[-1], *img_shape[:2])
    else:
        img_shape = data["train_x"][0, 0].flatten().shape

    def mk(key, s):
        x = data[key]
        if device is not None:
            return DeviceDataIterator(x, x.shape[1:2] + img_shape, device, seed=s, rank=rank, world=world)
        return DataIterator(X=x.astype(np.float32).reshape(x.shape[:2] + img_shape) / 255, seed=s, rank=rank,
                            world=world)

    return (mk("train_x", seed), mk("valid_x", None if seed is None else seed + 1),
            mk("test_x", None if seed is None else seed + 2))
