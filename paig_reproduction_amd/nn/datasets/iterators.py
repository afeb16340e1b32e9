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
    paig_gather_u8_f32; ``X`` is the device uint8 tensor (``X.shape[0]`` is N).

    The epoch permutation is drawn on the host exactly as DataIterator draws it
    (same RNG calls, same batches) and uploaded once per epoch; a batch is then
    a slice of that device permutation, so a step issues no host-to-device
    copy at all, only the gather launch.  ``out`` (next_batch / gather_into)
    lets a caller gather into a fixed buffer, e.g. the input of a captured
    HIP graph.

    bind_targets(xbuf, head_frames) makes the decoders read their targets as
    the dataset's bytes (ByteTargets): gathers into xbuf then convert only the
    first head_frames frames of every sequence (the encoder's input) and
    record the batch's dataset rows for the decoders."""

    def __init__(self, X_u8, shape, device, seed=None, rank=0, world=1):
        import torch
        self.shape = tuple(int(d) for d in shape)
        self.row = int(np.prod(X_u8.shape[1:]))
        assert self.row == int(np.prod(self.shape)), (X_u8.shape, shape)
        self.device = torch.device(device)
        self.idx_d = None
        self.bound = None
        super().__init__(torch.from_numpy(np.ascontiguousarray(X_u8)).to(self.device), None, seed, rank, world)

    def reset_iteration(self):
        import torch
        super().reset_iteration()
        # stream-ordered upload of this epoch's permutation (gathers of the
        # previous epoch that are still queued read their own buffer)
        self.idx_d = torch.from_numpy(self.indices.astype(np.int64)).pin_memory().to(self.device, non_blocking=True)

    def bind_targets(self, xbuf, head_frames):
        """Bind the fixed input buffer ``xbuf`` [B, *shape]: see ByteTargets.
        Returns the binding for ``Engine.byte_targets``."""
        self.bound = ByteTargets(self, xbuf, head_frames)
        return self.bound

    def _launch(self, idx_ptr, n, out):
        from paig_reproduction_amd._lib import lib, stream_handle
        if n:
            bt = self.bound
            if bt is not None and out.data_ptr() == bt.x_ptr:
                assert n == bt.B, (n, bt.B)
                lib().paig_gather_u8_f32_ex(self.X.data_ptr(), idx_ptr, out.data_ptr(), int(n), self.row, bt.head,
                                            bt.idx.data_ptr(), stream_handle(self.device))
            else:
                lib().paig_gather_u8_f32(self.X.data_ptr(), idx_ptr, out.data_ptr(), int(n), self.row,
                                         stream_handle(self.device))
        return out

    def _out(self, n, out):
        import torch
        if out is None:
            return torch.empty((n,) + self.shape, device=self.device)
        assert out.is_contiguous() and out.dtype == torch.float32 and tuple(out.shape) == (n,) + self.shape, \
            (tuple(out.shape), out.dtype)
        return out

    def _gather(self, idx, out=None):
        """Rows ``idx`` (host indices) -> float32 [len(idx), *shape]."""
        import torch
        idx = np.asarray(idx, dtype=np.int64)
        assert idx.size == 0 or (idx.min() >= 0 and idx.max() < self.num_examples)
        out = self._out(idx.size, out)
        if idx.size:
            idx_d = torch.from_numpy(idx).pin_memory().to(self.device, non_blocking=True)
            self._launch(idx_d.data_ptr(), idx.size, out)
        return out

    def next_batch(self, batch_size, data_type="train", shuffle=True, out=None):
        assert data_type in ["train", "val", "test"], "data_type must be 'train', 'val', or 'test'."
        # the same bookkeeping as DataIterator._take, on the device permutation
        lo = self.start_idx + self.rank * batch_size
        n = max(0, min(batch_size, self.num_examples - lo))
        idx_d = self.idx_d
        out = self._out(n, out)
        self._launch(idx_d.data_ptr() + 8 * lo, n, out)
        self._take(batch_size)   # advances start_idx / epoch (may upload the next permutation)
        return out, None

    def sample_random_batch(self, batch_size):
        np.random.randint(0, self.num_examples - batch_size)   # reference quirk (iterators.py:42-47)
        return self._gather(np.arange(self.start_idx, min(self.start_idx + batch_size, self.num_examples))), None


class ByteTargets:
    """The decoders' targets read from the device-resident dataset (SURVEY §8
    F2 + the fused SSE): a batch gathered into the bound buffer ``xbuf``
    converts only its first ``head_frames`` frames to float32 (what the
    encoder reads; the later frames of xbuf are NOT written), saves the
    batch's dataset rows in ``idx``, and the engine's rollout decoders
    (forward SSE and backward) read frame t of sequence b as X[idx[b]]
    bytes / 255 -- bit-identical to the float32 frame the full gather writes
    (paig_decoder_fwd_t8 / paig_decoder_bwd_t8).  Per sequence of T frames
    this drops the (T - head) float32 frames' write and re-read and reads
    every rollout target at 1 byte a value instead of 4 (the reconstruction
    decoders read the encoder's float32 frames, which are gathered anyway).

    The binding is a promise that only this iterator fills ``xbuf`` (a batch
    written into it otherwise would be decoded against stale rows) and that
    nothing reads its frames >= head_frames (model.input's tail).  The engine
    uses it for an input whose storage is ``xbuf``'s and whose shape matches."""

    SHAPES = ((2, 32), (3, 36), (2, 64))   # (objects, frame side) of the byte-target kernels

    def __init__(self, it, xbuf, head_frames):
        import torch
        assert xbuf.is_contiguous() and xbuf.dtype == torch.float32 and xbuf.device == it.device
        assert tuple(xbuf.shape[1:]) == it.shape, (tuple(xbuf.shape), it.shape)
        self.it = it
        self.B, self.T = int(xbuf.shape[0]), int(it.shape[0])
        self.frame = it.row // self.T
        self.head_frames = int(head_frames)
        assert 0 < self.head_frames <= self.T
        head = self.head_frames * self.frame
        self.head = min(it.row, -(-head // 16) * 16)   # the gather moves 16-byte multiples
        self.x_ptr = xbuf.data_ptr()
        self.base = it.X.data_ptr()
        self.idx = torch.zeros(self.B, dtype=torch.int64, device=it.device)
        self.idx_ptr = self.idx.data_ptr()

    def covers(self, x, lay):
        """True when the engine may decode ``x`` (layout ``lay``) against the
        bytes: x is the bound buffer and the frames it converts cover the
        encoder's."""
        return (x.data_ptr() == self.x_ptr and x.shape[0] == self.B and x.shape[1] == self.T and
                lay.frame == self.frame and lay.Te <= self.head_frames and (lay.K, lay.H) in self.SHAPES)


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
