"""the device-resident dataset yields exactly the batches of the
reference-semantics host iterator (same seed -> same permutation, drop-last,
rank sharding, uint8/255 with the Q5 reshape), bit for bit."""
import numpy as np
import pytest
import torch

from paig_reproduction_amd.nn.datasets.iterators import ByteTargets, DataIterator, DeviceDataIterator


def _data(n=23, T=5, H=8, C=3, seed=0):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(n, T, H, H, C), dtype=np.uint8)


def test_take_is_drop_last_and_sharded():
    X = np.zeros((10, 1), np.float32)
    it = DataIterator(X, seed=1, rank=1, world=2)
    seen = []
    while it.get_epoch() < 1:
        seen.append(it._take(2))
    assert len(seen) == 2 and all(len(s) == 2 for s in seen)   # 10 // (2*2) = 2 global batches


@pytest.mark.gpu
@pytest.mark.parametrize("rank,world", [(0, 1), (1, 2)])
def test_device_batches_match_host(rank, world):
    u8 = _data()
    N, T, H, W, C = u8.shape
    host = DataIterator(u8.astype(np.float32).reshape(N, T, C, H, W) / 255, seed=5, rank=rank, world=world)
    dev = DeviceDataIterator(u8, (T, C, H, W), "cuda:0", seed=5, rank=rank, world=world)
    for _ in range(12):                    # crosses epoch boundaries
        hx, _ = host.next_batch(3)
        dx, _ = dev.next_batch(3)
        torch.cuda.synchronize()
        assert dx.dtype == torch.float32 and tuple(dx.shape) == (3, T, C, H, W)
        assert np.array_equal(dx.cpu().numpy(), hx.astype(np.float32))
        assert host.get_epoch() == dev.get_epoch()


@pytest.mark.gpu
def test_gather_every_byte_value():
    """v / 255 of every byte value bit for bit as numpy's float32 division."""
    N, T, H, W, C = 4, 2, 8, 8, 3
    u8 = (np.arange(N * T * H * W * C) % 256).astype(np.uint8).reshape(N, T, H, W, C)
    want = u8.astype(np.float32).reshape(N, T, C, H, W) / 255
    dev = DeviceDataIterator(u8, (T, C, H, W), "cuda:0", seed=0)
    for _ in range(2):
        dx, _ = dev.next_batch(2)
        torch.cuda.synchronize()
        for row in dx.cpu().numpy():
            assert any(np.array_equal(row, w) for w in want)
    dx = torch.empty(N, T, C, H, W, device="cuda:0")
    dev.reset_iteration()
    dev.next_batch(N, out=dx)
    torch.cuda.synchronize()
    assert sorted(map(bytes, dx.cpu().numpy())) == sorted(map(bytes, want))   # all 256 values, every sequence


def test_byte_targets_binding_rules():
    """ByteTargets (CPU-side bookkeeping only): the gathered head rounds up to
    16-byte multiples within the row, and the engine may use the bytes only
    for the bound buffer with a matching layout and an encoder within the head."""
    from types import SimpleNamespace
    u8 = _data(n=6, T=5, H=6, C=3)            # frame 108 bytes
    N, T, H, W, C = u8.shape
    # the iterator's fields ByteTargets reads (a DeviceDataIterator needs a GPU)
    it = SimpleNamespace(shape=(T, C, H, W), row=T * C * H * W, device=torch.device("cpu"),
                         X=torch.from_numpy(u8))
    xbuf = torch.empty((2, T, C, H, W))
    bt = ByteTargets(it, xbuf, 3)
    assert bt.frame == C * H * W and bt.head == 336 and bt.head % 16 == 0 and bt.head <= it.row
    assert bt.base == it.X.data_ptr() and tuple(bt.idx.shape) == (2,) and bt.idx.dtype == torch.int64
    lay = SimpleNamespace(frame=bt.frame, Te=3, K=2, H=32)
    assert bt.covers(xbuf, lay)
    assert not bt.covers(torch.empty_like(xbuf), lay)                      # another buffer
    assert not bt.covers(xbuf, SimpleNamespace(frame=bt.frame, Te=4, K=2, H=32))   # encoder past the head
    assert not bt.covers(xbuf, SimpleNamespace(frame=bt.frame, Te=3, K=3, H=32))   # no byte-target kernel
    assert ByteTargets(it, xbuf, T).head == it.row
