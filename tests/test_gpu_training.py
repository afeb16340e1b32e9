"""Training-loop and test-phase parity with the reference, against fixtures the
reference's own loop produced (tests/golden/train_*.npz, gen_golden_train.py):

* a 10-step RMSprop trajectory (nn/network/base.py:134-160, fresh loss);
* the reference's actual step, quirk Q1 (--loss_mode reference: the loss reads
  the stale output of the last eval forward, base.py:141-143 vs :195);
* the test phase at test_seq_len (runners/torch_run_physics.py:101-117,
  eval_performance base.py:174-218);
* Adam / SGD / momentum / RMSprop (base.py:12-17) against torch.optim on the
  same gradients.

RMSprop trajectories are ill-conditioned: its first update is about
lr * sign(g) / sqrt(1 - alpha) whatever |g| is, so gradients that are pure
rounding noise (near-cancelling sums) take full-size steps of either sign, and
max-pool / ReLU decisions then flip.  Even the fp32 oracle (the same CPU aten
ops as the reference) ends 10 steps with parameters far from the reference's.
So the trajectory bar is an envelope: the HIP run may sit no further from the
reference than ENVELOPE_K times the furthest of an ensemble of honest fp32 runs
(the oracle on one-ulp-perturbed weights), computed in the test.  Step 0 (no
update yet) is held to the fixed 1e-4 bar.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from helpers import GOLDEN_DIR, golden_weights, rel_err, grad_checks, RTOL
from envelope import ENVELOPE_K, _ulp_perturbed
from oracle import physics_oracle as O

pytestmark = pytest.mark.gpu

TRAJ_ENSEMBLE = 3
# chaotic 3-body rollout at test_seq_len 40: measured 9.3e-7 (output_seq) /
# 5.8e-7 (pos_vel_seq) against the fixture; the parity tests' 1e-5 bar
ROLLOUT_RTOL_3BP = 1e-5


def _load(name):
    return np.load(os.path.join(GOLDEN_DIR, f"train_{name}.npz"), allow_pickle=False)


def _model(z, dev):
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet
    task, cell, seq_len, ins, pred, size, B, ae, alt = [str(s) for s in z["config"]]
    torch.manual_seed(0)
    m = PhysicsNet(task, 100, 1, cell, int(seq_len), int(ins), int(pred), float(ae), bool(int(alt)), True,
                   int(size) ** 2, "conv_encoder", "conv_st_decoder", device=dev).to(dev)
    m.load_state_dict({k: v.to(dev) for k, v in golden_weights(z).items()})
    return m


def _x(u8, dev=None):
    x = O.input_from_u8(u8)
    return x.to(dev) if dev is not None else x


def _final_vector(z, params, keys):
    """The fixture's stored final values (full small tensors, 64x64 slices of
    the big ones) and the same entries of ``params`` -> two flat vectors."""
    a, b = [], []
    for k in keys:
        v = params[k].detach().double().cpu().numpy()
        if "final/" + k in z.files:
            a.append(v.reshape(-1))
            b.append(np.asarray(z["final/" + k], dtype=np.float64).reshape(-1))
        else:
            a.append(v.reshape(v.shape[0], -1)[:64, :64].reshape(-1))
            b.append(np.asarray(z["finalslice/" + k], dtype=np.float64).reshape(-1))
    return np.concatenate(a), np.concatenate(b)


def _l2rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("name", ["spring_s12", "mnist_s12"])
def test_rmsprop_trajectory(name):
    dev = torch.device("cuda:0")
    z = _load("traj_" + name)
    steps, lr = int(z["steps"]), float(z["lr"])
    ref_losses = np.asarray(z["losses"])
    m = _model(z, dev)
    m.build_optimizer(lr, "rmsprop", True)
    xs = [_x(z["input_u8_0"], dev), _x(z["input_u8_1"], dev)]
    losses = []
    for s in range(steps):
        m.output = m(xs[s % 2])
        tl, (p, e, r) = m.compute_loss()
        losses.append([float(v.detach()) for v in (tl, p, e, r)])
        m.optimizer.zero_grad(set_to_none=True)
        tl.backward()
        m.optimizer.step()
    torch.cuda.synchronize()
    losses = np.array(losses)
    cfg, _ = O.cfg_from_golden(z)
    state = golden_weights(z)
    keys = list(O.live_params(state, cfg))
    hip_vec, ref_vec = _final_vector(z, dict(m.named_parameters()), keys)
    init_vec, _ = _final_vector(z, state, keys)
    # step 0 precedes any update: the fixed bar
    assert rel_err(losses[0], ref_losses[0]) <= RTOL, (losses[0], ref_losses[0])
    # the honest-fp32 ensemble
    torch.set_num_threads(8)
    xs_cpu = [_x(z["input_u8_0"]), _x(z["input_u8_1"])]
    ens_loss, ens_par = [], []
    for seed in range(TRAJ_ENSEMBLE):
        L, S = O.train_trajectory(_ulp_perturbed(state, seed), cfg, xs_cpu, lr, steps)
        ens_loss.append(rel_err(np.array(L), ref_losses))
        a, b = _final_vector(z, S, keys)
        ens_par.append(_l2rel(a - init_vec, b - init_vec))
    e_loss = rel_err(losses, ref_losses)
    e_par = _l2rel(hip_vec - init_vec, ref_vec - init_vec)   # distance of the 10-step parameter updates
    print(name, f"loss {e_loss:.2e} (fp32 ensemble max {max(ens_loss):.2e}); update {e_par:.2e} "
                f"(ensemble max {max(ens_par):.2e})")
    assert e_loss <= max(ENVELOPE_K * max(ens_loss), 1e-5), (e_loss, ens_loss)
    assert e_par <= max(ENVELOPE_K * max(ens_par), 1e-4), (e_par, ens_par)


def test_reference_loss_mode():
    """Quirk Q1 exactly as the reference's loop does it: an eval forward under
    no_grad leaves self.output; the train steps' loss reads it (pred/extrap
    constant), only the reconstruction term carries gradient, and the rollout
    branch's parameters get no gradient at all."""
    dev = torch.device("cuda:0")
    z = _load("refmode_spring_s12")
    m = _model(z, dev)
    m.loss_mode = "reference"
    m.build_optimizer(float(z["lr"]), "rmsprop", True)
    with torch.no_grad():
        m.output = m.conv_feedforward(_x(z["input_u8_eval"], dev))
    losses = []
    for s in range(2):
        m.forward(_x(z["input_u8_%d" % s], dev))    # result discarded (base.py:142)
        tl, (p, e, r) = m.compute_loss()
        losses.append([float(v.detach()) for v in (tl, p, e, r)])
        m.optimizer.zero_grad(set_to_none=True)
        tl.backward()
        if s == 0:
            grads = {k: q.grad for k, q in m.named_parameters() if q.grad is not None}
            assert sorted(grads) == sorted(str(k) for k in z["grad_keys"]), \
                set(grads) ^ set(str(k) for k in z["grad_keys"])
            gerr = grad_checks(z, grads, 1e9)
            # this fixture sits on a near-tie max-pool decision: 4 of 6 one-ulp
            # perturbations of the weights move the early U-Net gradients by
            # ~5e-3 (measured); the bar is the fp32 envelope, at least 1e-4
            cfg, _ = O.cfg_from_golden(z)
            state = golden_weights(z)
            torch.set_num_threads(8)
            xe, x0 = _x(z["input_u8_eval"]), _x(z["input_u8_0"])
            ens = [grad_checks(z, O.reference_mode_steps(_ulp_perturbed(state, sd), cfg, xe, [x0],
                                                         float(z["lr"]))[1], 1e9) for sd in range(4)]
            over = {k: (v, max(ENVELOPE_K * max(e[k] for e in ens), RTOL)) for k, v in gerr.items()
                    if v > max(ENVELOPE_K * max(e[k] for e in ens), RTOL)}
            print("refmode worst grad", max(gerr.items(), key=lambda kv: kv[1]))
            assert not over, over
        m.optimizer.step()
    torch.cuda.synchronize()
    ref = np.asarray(z["losses"])
    assert rel_err(np.array(losses[0]), ref[0]) <= RTOL, (losses[0], ref[0])
    # the second step follows one RMSprop update of the encoder/decoder
    assert rel_err(np.array(losses[1]), ref[1]) <= 1e-3, (losses[1], ref[1])


@pytest.mark.parametrize("name", ["spring_s30", "3bp_s40"])
def test_eval_test_phase(name):
    """The test phase: a model built at test_seq_len, eval_performance over a
    test set of fewer than 100 sequences (one whole-set batch, Q15)."""
    from paig_reproduction_amd.nn.datasets.iterators import DataIterator
    dev = torch.device("cuda:0")
    z = _load("eval_" + name)
    m = _model(z, dev)
    m.extra_valid_fns.clear()   # visualisation (moviepy in the reference), cleared for the fixture too
    m.extra_test_fns.clear()
    x = _x(z["input_u8"])
    m.test_iterator = DataIterator(x.numpy(), seed=0)
    m.build_optimizer(1e-3, "rmsprop", True)
    with tempfile.TemporaryDirectory() as d:
        m.save_dir = d
        metrics = m.eval_performance(100, type="test")
        assert os.path.exists(os.path.join(d, "outputs.npz"))
    rt = ROLLOUT_RTOL_3BP if name.startswith("3bp") else RTOL
    errs = {}
    for k in ("eval_pred_loss", "eval_extrap_loss", "eval_recons_loss"):
        bar = RTOL if k == "eval_recons_loss" else rt
        e = errs[k] = rel_err(np.asarray(metrics[k], dtype=np.float64).reshape(()), z["metric/" + k])
        assert e <= bar, (k, e, float(metrics[k]), float(z["metric/" + k]))
    with torch.no_grad():
        out = m.conv_feedforward(x.to(dev))
    torch.cuda.synchronize()
    errs["output_seq"] = rel_err(out, z["output_seq"])
    errs["pos_vel_seq"] = rel_err(m.pos_vel_seq, z["pos_vel_seq"])
    print(name, "eval vs fixture:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["output_seq"] <= rt
    assert errs["pos_vel_seq"] <= rt


@pytest.mark.parametrize("kind", ["adam", "sgd", "momentum", "rmsprop"])
def test_optimizer_matches_torch(kind):
    """FlatOptimizer (one fused kernel per dtype) vs torch.optim with the
    reference's constructor arguments (base.py:12-17), 3 steps on the same
    gradients, fp32 and the fp64 physics parameters."""
    dev = torch.device("cuda:0")
    from helpers import load_golden
    z = load_golden("spring_s12")
    m = _model(z, dev)
    m.build_optimizer(1e-3, kind, True)
    m.output = m(_x(z["input_u8"], dev))
    tl, _ = m.compute_loss()
    m.optimizer.zero_grad(set_to_none=True)
    tl.backward()
    torch.cuda.synchronize()
    named = {k: p for k, p in m.named_parameters() if p.grad is not None}
    ref = {k: torch.nn.Parameter(p.detach().clone()) for k, p in named.items()}
    for k, p in ref.items():
        p.grad = named[k].grad.detach().clone()
    make = {"adam": lambda ps: torch.optim.Adam(ps, lr=1e-3), "rmsprop": lambda ps: torch.optim.RMSprop(ps, lr=1e-3),
            "momentum": lambda ps: torch.optim.SGD(ps, momentum=0.9, lr=1e-3),
            "sgd": lambda ps: torch.optim.SGD(ps, lr=1e-3)}[kind]
    topt = make(list(ref.values()))
    for _ in range(3):
        topt.step()
        m.optimizer.step()
    torch.cuda.synchronize()
    for k, p in named.items():
        e = rel_err(p.detach(), ref[k].detach())
        assert e <= 2e-6, (kind, k, e)   # Adam's sqrt / bias correction round differently by an ulp


@pytest.mark.parametrize("kind", ["rmsprop", "adam", "momentum"])
def test_optimizer_skips_params_without_grad(kind):
    """torch semantics after zero_grad(set_to_none=True): a full
    step, zero_grad, then a standalone encoder backward (only the encoder's
    parameters get gradients) and optimizer.step(): exactly the encoder's
    parameters move, as torch.optim moves them from the same gradients and
    state; every other parameter (whose flat gradient slot still holds the
    previous step's values) stays put.  Then a fused step accumulates onto
    the encoder grads only."""
    dev = torch.device("cuda:0")
    from helpers import load_golden
    z = load_golden("spring_s12")
    m = _model(z, dev)
    m.build_optimizer(1e-3, kind, True)
    x = _x(z["input_u8"], dev)
    make = {"adam": lambda ps: torch.optim.Adam(ps, lr=1e-3), "rmsprop": lambda ps: torch.optim.RMSprop(ps, lr=1e-3),
            "momentum": lambda ps: torch.optim.SGD(ps, momentum=0.9, lr=1e-3)}[kind]
    # step 1: full backward (every live parameter has a gradient)
    m.output = m(x)
    tl, _ = m.compute_loss()
    m.optimizer.zero_grad(set_to_none=True)
    tl.backward()
    torch.cuda.synchronize()
    named = {k: p for k, p in m.named_parameters() if p.grad is not None}
    ref = {k: torch.nn.Parameter(p.detach().clone()) for k, p in named.items()}
    for k, p in ref.items():
        p.grad = named[k].grad.detach().clone()
    topt = make(list(ref.values()))
    topt.step()
    m.optimizer.step()
    # step 2: standalone encoder call, only encoder.* get gradients
    m.optimizer.zero_grad(set_to_none=True)
    topt.zero_grad(set_to_none=True)
    frames = x[:, :m.input_steps + m.pred_steps].reshape(-1, 3, 32, 32)
    pos, _, _ = m.encoder(frames)
    pos.sum().backward()
    torch.cuda.synchronize()
    enc = [k for k, p in named.items() if p.grad is not None]
    assert enc and all(k.startswith("encoder.") for k in enc)
    assert all(named[k].grad is None for k in named if not k.startswith("encoder."))
    for k in enc:
        ref[k].grad = named[k].grad.detach().clone()
    before = {k: p.detach().clone() for k, p in named.items()}
    topt.step()
    m.optimizer.step()
    torch.cuda.synchronize()
    for k, p in named.items():
        if k in enc:
            assert rel_err(p.detach(), ref[k].detach()) <= 2e-6, (kind, k)
        else:
            assert torch.equal(p.detach(), before[k]), f"{kind}: {k} moved without a gradient"
    # step 3: a fused step onto the encoder's accumulated grads: the others
    # start from zero, not from their stale slots
    g_enc = {k: named[k].grad.detach().clone() for k in enc}
    m.output = m(x)
    tl, _ = m.compute_loss()
    tl.backward()
    torch.cuda.synchronize()
    m2 = _model(z, dev)
    with torch.no_grad():
        for (k, p), (k2, p2) in zip(m.named_parameters(), m2.named_parameters()):
            p2.copy_(p)
    m2.build_optimizer(1e-3, kind, True)
    m2.output = m2(x)
    tl2, _ = m2.compute_loss()
    tl2.backward()
    torch.cuda.synchronize()
    named2 = dict(m2.named_parameters())
    for k in named:
        want = named2[k].grad + (g_enc[k] if k in g_enc else 0)
        assert rel_err(named[k].grad, want) <= 1e-6, (kind, k)


def test_rollout_sse_second_gradient_path():
    """the live-steps hint that lets the rollout decoder backward
    skip the frames without a loss weight (physics_models.py:129-139 weights
    loss[:, :pred_steps] only) must not survive when the per-frame SSE gets a
    second gradient path that autograd accumulates into the same tensor:
    every rollout frame then carries a weight.  Gradients of
    train_loss + 0.5 * sum(sse_roll) must equal the sum of the two losses'
    separate gradients."""
    dev = torch.device("cuda:0")
    z = _load("traj_spring_s12")
    x = _x(z["input_u8_0"], dev)

    def grads(which):
        m = _model(z, dev)
        m.output = m(x)
        loss, _ = m.compute_loss()
        extra = 0.5 * m._sse_roll.sum()
        total = {"train": loss, "sse": extra, "both": loss + extra}[which]
        total.backward()
        return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}

    ga, gb, gc = grads("train"), grads("sse"), grads("both")
    assert set(gc) == set(ga) | set(gb)
    worst = 0.0
    for k in gc:
        want = ga.get(k, 0) + gb.get(k, 0)
        worst = max(worst, rel_err(gc[k], want))
    # the extrapolation frames' decoder gradient reaches the VFN sources: a
    # surviving mark would drop it entirely (an O(1) error)
    assert worst <= 1e-5, worst


def test_two_forwards_before_backward():
    """each grad-enabled forward owns the per-launch activation
    maxima its conv weight gradients are scaled by (the split arithmetic's
    X exponent).  Two forwards of the same shape -- the second on inputs 64x
    larger -- then ONE backward of the summed losses must give the sum of the
    two steps' separate gradients (a shared buffer would scale the first
    step's activations by the second's maxima)."""
    dev = torch.device("cuda:0")
    z = _load("traj_spring_s12")
    x1 = _x(z["input_u8_0"], dev)
    x2 = _x(z["input_u8_1"], dev) * 64.0

    def grads(xs):
        m = _model(z, dev)
        total = 0
        for x in xs:
            m.output = m(x)
            loss, _ = m.compute_loss()
            total = total + loss
        total.backward()
        return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}

    ga, gb, gc = grads([x1]), grads([x2]), grads([x1, x2])
    worst = max(rel_err(gc[k], ga[k] + gb[k]) for k in gc)
    assert worst <= 1e-5, worst
