"""Dataset iterators (reference nn/datasets/iterators.py:4-69).

Same semantics: unseeded shuffle per epoch (an optional ``seed`` makes it
reproducible), drop-last (the epoch ends when ``start + batch > N``), uint8/255
to float32, and quirk Q5 — NHWC frames are RESHAPED (not transposed) to
[C, H, W].  ``--datapoints`` is a no-op exactly as in the reference (Q7).

Data-parallel: ``rank``/``world`` give each rank a disjoint slice of every
epoch's shared permutation (a shared ``seed`` keeps the permutations equal).
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

    def next_batch(self, batch_size, data_type="train", shuffle=True):
        assert data_type in ["train", "val", "test"], "data_type must be 'train', 'val', or 'test'."
        gb = batch_size * self.world
        lo = self.start_idx + self.rank * batch_size
        idx = self.indices[lo:lo + batch_size]
        batch_x = self.X[idx]
        batch_y = self.Y[idx] if self.Y is not None else self.Y
        self.start_idx += gb
        if self.start_idx + gb > self.num_examples:
            self.reset_iteration()
            self.epochs_completed += 1
        return (batch_x, batch_y)

    def sample_random_batch(self, batch_size):
        # reference quirk kept: the drawn start_idx is unused (iterators.py:42-47)
        np.random.randint(0, self.num_examples - batch_size)
        batch_x = self.X[self.start_idx:self.start_idx + batch_size]
        batch_y = self.Y[self.start_idx:self.start_idx + batch_size] if self.Y is not None else self.Y
        return (batch_x, batch_y)


def get_iterators(file, conv=False, datapoints=0, seed=None, rank=0, world=1):
    data = np.load(file)
    if conv:
        img_shape = data["train_x"][0, 0].shape
        img_shape = (img_shape[-1], *img_shape[:2])
    else:
        img_shape = data["train_x"][0, 0].flatten().shape

    def mk(key, s):
        x = data[key]
        return DataIterator(X=x.astype(np.float32).reshape(x.shape[:2] + img_shape) / 255, seed=s, rank=rank,
                            world=world)

    return (mk("train_x", seed), mk("valid_x", None if seed is None else seed + 1),
            mk("test_x", None if seed is None else seed + 2))
