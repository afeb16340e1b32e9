"""Byte targets (DeviceDataIterator.bind_targets, paig_decoder_fwd_t8 /
paig_decoder_bwd_t8, paig_gather_u8_f32_ex): a training step whose decoders
read their targets as the dataset's bytes, and whose gather converts only the
encoder's frames, is bit-identical to the step on the fully gathered float32
batch -- outputs, the three losses, every parameter gradient and the RMSprop
update -- for every task shape bench.py runs, across epoch boundaries (the
decoders follow the permutation through the saved row indices).  The frames
the bound gather skips are poisoned with NaN: any read of them would show.
The same harness holds the merged launches (the rollout + reconstruction
decode, paig_decoder_fwd_rollout; the weight prep + first conv,
paig_conv_wprep_defer) to their separate forms, bit for bit.
"""
import os

import numpy as np
import pytest
import torch

from paig_reproduction_amd.nn.datasets.iterators import DeviceDataIterator

pytestmark = pytest.mark.gpu

# task: (cell, ins, pred, size) -- bench.py TASKS
TASKS = {"spring_color": ("spring_ode_cell", 4, 6, 32), "bouncing_balls": ("bouncing_ode_cell", 4, 6, 32),
         "3bp_color": ("gravity_ode_cell", 4, 12, 36), "mnist_spring_color": ("spring_ode_cell", 3, 7, 64)}
OUT_KEYS = ("output", "recons_out", "pos_vel_seq", "enc_pos")


def _run(task, byte_targets, steps=3, B=6, N=14, extrap=4, merge=True):
    from paig_reproduction_amd.nn.datasets.synth import render_sequences
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet
    from paig_reproduction_amd.graph_step import GraphStep
    dev = torch.device("cuda:0")
    cell, ins, pred, size = TASKS[task]
    T = ins + pred + extrap
    torch.manual_seed(0)
    m = PhysicsNet(task, 100, 1, cell, T, ins, pred, 3.0, False, True, size * size, "conv_encoder",
                   "conv_st_decoder", device=dev).to(dev)
    m.build_optimizer(1e-3, "rmsprop", True)
    u8 = render_sequences(task, N, T, seed=7)
    it = DeviceDataIterator(u8, (T, 3, size, size), dev, seed=2)
    xbuf = torch.full((B, T, 3, size, size), float("nan"), device=dev)
    gs = GraphStep(m, xbuf, 1, graph=False)
    if byte_targets:
        gs.eng.byte_targets = it.bind_targets(xbuf, ins + pred)
    rec = []
    knobs = ("PAIG_MERGE_ROLL", "PAIG_WPREP_MERGE", "PAIG_GEMM_EPI_MERGE", "PAIG_LOSSW_INKERNEL")   # merged forms, or the A/B ones
    old_env = {k: os.environ.get(k) for k in knobs}
    for k in knobs:
        os.environ[k] = "1" if merge else "0"
    try:
        for s in range(steps):   # N=14, B=6: the third batch opens a new epoch (a new permutation)
            rec.append(_step(m, gs, it, xbuf, B, ins, pred, byte_targets))
    finally:
        for k, v in old_env.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    r = {"param:" + n: p.detach().clone() for n, p in m.named_parameters()}
    rec.append(r)
    return rec, it.get_epoch()


def _step(m, gs, it, xbuf, B, ins, pred, byte_targets):
    it.next_batch(B, out=xbuf)
    loss = gs.eager()
    torch.cuda.synchronize()
    r = {k: getattr(m, k).detach().clone() for k in OUT_KEYS}
    r.update(loss=loss.detach().clone(), extrap=m.extrap_loss.detach().clone(), recons=m.recons_loss.detach().clone(),
             xhead=xbuf[:, :ins + pred].clone())
    r.update({"grad:" + n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None})
    if byte_targets:
        r["tail_nan"] = bool(torch.isnan(xbuf[:, ins + pred:]).all())
    return r


def _same(a, b):
    return a.shape == b.shape and bool(torch.equal(torch.nan_to_num(a, 7.0), torch.nan_to_num(b, 7.0))) and \
        bool((torch.isnan(a) == torch.isnan(b)).all())


@pytest.mark.parametrize("task", list(TASKS))
def test_byte_targets_step_bit_identical(task):
    ref, ep_ref = _run(task, False)
    got, ep_got = _run(task, True)
    assert ep_ref == ep_got >= 1
    assert len(ref) == len(got)
    for s, (a, b) in enumerate(zip(ref, got)):
        assert set(a) - {"tail_nan"} == set(b) - {"tail_nan"}, (s, set(a) ^ set(b))
        bad = [k for k in a if k != "tail_nan" and not _same(a[k], b[k])]
        assert not bad, f"step {s}: {bad[:8]}"
        if "tail_nan" in b:
            assert b["tail_nan"], f"step {s}: the bound gather wrote frames past the encoder's"
    assert np.isfinite(float(got[-2]["loss"]))


@pytest.mark.parametrize("task", list(TASKS))
def test_merged_launches_bit_identical(task):
    """paig_decoder_fwd_rollout (the rollout and the reconstruction decode in
    one launch), paig_conv_wprep_defer (the weight prep in the first conv's
    launch, whose weights are then staged in-kernel) and the dense weight
    gradients' deferred split-K epilogues (paig_gemm_defer_epilogue) give the
    separate launches' step bit for bit."""
    ref, _ = _run(task, True, merge=False)
    got, _ = _run(task, True, merge=True)
    for s, (a, b) in enumerate(zip(ref, got)):
        bad = [k for k in a if k != "tail_nan" and not _same(a[k], b[k])] if set(a) == set(b) else sorted(set(a) ^ set(b))
        assert not bad, f"step {s}: {bad[:8]}"


def test_byte_targets_unbound_buffer_uses_float_frames():
    """An input that is not the bound buffer decodes against its own frames."""
    from paig_reproduction_amd.nn.datasets.synth import render_sequences
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet
    dev = torch.device("cuda:0")
    cell, ins, pred, size = TASKS["spring_color"]
    T, B = 12, 4
    u8 = render_sequences("spring_color", 8, T, seed=3)
    torch.manual_seed(0)
    m = PhysicsNet("spring_color", 100, 1, cell, T, ins, pred, 3.0, False, True, size * size, "conv_encoder",
                   "conv_st_decoder", device=dev).to(dev)
    it = DeviceDataIterator(u8, (T, 3, size, size), dev, seed=1)
    xbuf = torch.empty((B, T, 3, size, size), device=dev)
    eng = m._native()
    eng.byte_targets = it.bind_targets(xbuf, ins + pred)
    other = torch.empty_like(xbuf)
    it.next_batch(B, out=other)            # full gather (not the bound buffer)
    sse = []
    with torch.no_grad():
        for bound in (True, False):
            if not bound:
                eng.byte_targets = None
            m(other)
            sse.append(torch.cat([m._sse_rec, m._sse_roll]).clone())
    torch.cuda.synchronize()
    # (the bound buffer's row indices are all 0: decoding against them would differ)
    assert torch.equal(sse[0], sse[1])
    assert bool(torch.isfinite(other).all())
