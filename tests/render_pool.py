"""Whole batches of DISTINCT synthetic sequences for the full-size GPU tests
(a batch tiled from 64 or 128 rendered sequences cannot
show an error that aliases sequence i with i + 64k).

The renderer (paig_reproduction_amd/nn/datasets/synth.py) is a per-sequence
Python loop (bouncing B=1024 x 100 frames takes ~70 s on one core), so the
batch is rendered in chunks, each from its own seed, in a pool of fresh
interpreter processes (spawn: nothing of the parent's GPU state is shared).
The chunks' seeds differ, so no two sequences of a batch coincide.
"""
import functools
import os
from concurrent.futures import ProcessPoolExecutor
import multiprocessing as mp

import numpy as np


def _chunk(args):
    task, n, seq_len, seed = args
    from paig_reproduction_amd.nn.datasets.synth import render_sequences
    return render_sequences(task, n, seq_len, seed=seed)


@functools.lru_cache(maxsize=8)
def render_distinct(task, n, seq_len, seed, chunk=32, workers=None):
    """uint8 [n, seq_len, H, W, 3]: n sequences, chunk i rendered with seed
    seed * 100003 + i (cached: the parametrised tests share batches; the
    array is read-only)."""
    jobs = [(task, min(chunk, n - i), seq_len, seed * 100003 + i // chunk) for i in range(0, n, chunk)]
    workers = workers or max(1, min(16, len(os.sched_getaffinity(0)), len(jobs)))
    if workers == 1:
        parts = [_chunk(j) for j in jobs]
    else:
        with ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn")) as ex:
            parts = list(ex.map(_chunk, jobs))
    u8 = np.concatenate(parts, 0)
    assert u8.shape[0] == n
    u8.setflags(write=False)
    return u8
