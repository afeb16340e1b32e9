"""Host-side data path, CPU only.

Reference semantics checked here (``nn/datasets/iterators.py``):
* ``get_iterators`` casts uint8/255 to float32 and RESHAPES NHWC -> [C,H,W]
  without transposing (quirk Q5, ``iterators.py:60-67``);
* ``next_batch`` walks a shuffled permutation and drops the ragged tail
  (``iterators.py:26-40``);
* data-parallel sharding: the ranks of one global batch take disjoint slices
  of the same permutation and together cover it.
The synthetic renderer stands in for the reference's dataset files (which
do not ship), so it is checked for layout and determinism only.
"""
import numpy as np
import pytest

from paig_reproduction_amd.nn.datasets.iterators import DataIterator, get_iterators
from paig_reproduction_amd.nn.datasets.synth import TASKS, as_model_input, render_sequences, write_dataset


def test_get_iterators_reshapes_not_transposes(tmp_path):
    path = write_dataset(str(tmp_path / "d.npz"), "spring_color", 6, 5, 3, 3, seed=2)
    raw = np.load(path)["train_x"]
    tr, va, te = get_iterators(path, conv=True, seed=7)
    assert tr.X.shape == (5, 6, 3, 32, 32) and tr.X.dtype == np.float32
    assert np.array_equal(tr.X, raw.astype(np.float32).reshape(5, 6, 3, 32, 32) / 255)
    assert np.array_equal(tr.X, as_model_input(raw))
    # a transpose would differ for any non-constant frame
    assert not np.array_equal(tr.X, raw.astype(np.float32).transpose(0, 1, 4, 2, 3) / 255)
    assert va.X.shape[0] == 3 and te.X.shape[0] == 3
    flat, _, _ = get_iterators(path, conv=False, seed=7)
    assert flat.X.shape == (5, 6, 32 * 32 * 3)


@pytest.mark.parametrize("n,b", [(10, 3), (12, 4), (7, 7), (5, 6)])
def test_epoch_is_a_permutation_with_drop_last(n, b):
    X = np.arange(n, dtype=np.float32)[:, None]
    it = DataIterator(X, seed=3)
    seen = []
    while it.get_epoch() < 1 and len(seen) < 100:
        bx, _ = it.next_batch(b)
        seen.append(bx[:, 0].astype(int))
    if b > n:                                    # reference: every batch is ragged -> epoch ends at once
        assert it.get_epoch() == 1
        return
    assert len(seen) == n // b and all(len(s) == b for s in seen)
    allidx = np.concatenate(seen)
    assert len(np.unique(allidx)) == len(allidx)   # no repeats inside an epoch


def test_rank_shards_cover_the_global_batch():
    n, b, world = 40, 4, 4
    X = np.arange(n, dtype=np.float32)[:, None]
    its = [DataIterator(X, seed=11, rank=r, world=world) for r in range(world)]
    ref = DataIterator(X, seed=11)
    for _ in range(6):                           # crosses an epoch boundary (40 // 16 = 2 batches/epoch)
        parts = [it.next_batch(b)[0][:, 0] for it in its]
        whole = ref.next_batch(b * world)[0][:, 0]
        assert np.array_equal(np.concatenate(parts), whole)
        assert len({int(v) for p in parts for v in p}) == b * world
    assert len({it.get_epoch() for it in its}) == 1


def test_seeded_iterators_are_reproducible():
    X = np.arange(50, dtype=np.float32)[:, None]
    a, b = DataIterator(X, seed=5), DataIterator(X, seed=5)
    for _ in range(10):
        assert np.array_equal(a.next_batch(7)[0], b.next_batch(7)[0])


@pytest.mark.parametrize("task", sorted(TASKS))
def test_renderer_layout_and_determinism(task):
    n_objs, size, _ = TASKS[task]
    u8 = render_sequences(task, 2, 5, seed=4)
    assert u8.shape == (2, 5, size, size, 3) and u8.dtype == np.uint8
    assert np.array_equal(u8, render_sequences(task, 2, 5, seed=4))
    assert u8.max() > 0
    # object j lives on channel 2 - (j % 3): with fewer than 3 objects channel 0 stays empty
    if n_objs < 3 and task != "mnist_spring_color":
        assert u8[..., 0].max() == 0


def test_render_distinct_batches_have_no_repeats():
    """The full-size GPU tests' batches (tests/render_pool.py): every
    sequence distinct, deterministic per seed, chunked over a spawn pool."""
    from render_pool import render_distinct
    a = render_distinct("spring_color", 40, 6, 7, chunk=8, workers=2)
    assert a.shape == (40, 6, 32, 32, 3) and a.dtype == np.uint8
    flat = a.reshape(40, -1)
    assert len({r.tobytes() for r in flat}) == 40
    b = render_distinct("spring_color", 40, 6, 7, chunk=8, workers=1)
    assert np.array_equal(a, b)
