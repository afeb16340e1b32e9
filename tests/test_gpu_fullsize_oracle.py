"""The 1e-4 parity bar at BASELINE.json's benched sizes (VERDICT r03 item 2,
r04 item 2): the CPU oracle (tests' checker, oracle/physics_oracle.py, pinned
to the reference's golden vectors) runs on the GPU box's host cores -- as
bench.py's cpu_baseline already does -- on every workload a bench line is
quoted on, WHOLE batches:

* config #1 spring_color B=100, seq_len 50 (4 in / 6 pred / 40 extrap), the
  headline workload;
* config #3 3bp_color B=512, seq 20 (36 x 36, gravity rollout);
* config #4 mnist_spring_color B=256, seq 12 (64 x 64, the UNet);
* config #5 bouncing_balls B=1024, seq 100 (96 rollout steps).

For each: the HIP step's outputs (latent positions, masks, reconstructions,
rollout frames, positions/velocities) and losses within 1e-4 normwise of the
fp32 oracle (north_star; 3bp's chaotic rollout at ROLLOUT_RTOL_3BP), and
EVERY parameter gradient element against the float64 oracle within
ENVELOPE_K x the spread of honest fp32 runs (the oracle on one-ulp-perturbed
weights), as tests/test_gpu_envelope.py does on the fixtures.  The measured
errors are printed (`pytest -s`) and quoted in DESIGN.md section 2.

Reference workload: runners/torch_run_physics.py:49-75 (presets),
nn/network/physics_models.py:119-142 (losses), :204-245 (forward).
"""
import numpy as np
import pytest
import torch

from envelope import ENVELOPE_FLOOR, ENVELOPE_K, _ulp_perturbed
from helpers import RTOL, rel_err
from oracle import physics_oracle as O

pytestmark = pytest.mark.gpu

OUT_KEYS = ("enc_pos", "enc_masks", "recons_out", "output_seq", "pos_vel_seq")
ENSEMBLE_FULL = 4
# 3bp's gravity rollout is chaotic: two fp32 CPU runs of the reference differ
# by 1.7e-5 on the fixture (test_oracle_golden); bar = ~3x the largest error
# measured on the fixture and at B=512
ROLLOUT_RTOL_3BP = 1e-5
# 3bp's velocities on their own scale: see tests/test_gpu_parity.py VEL_RTOL_3BP
VEL_RTOL_3BP = 5e-5


def _threads():
    import os
    n = len(os.sched_getaffinity(0))
    torch.set_num_threads(max(1, min(n, 16)))


def _model(task, cell, seq_len, ins, pred, size, B, seed=3):
    from paig_reproduction_amd.nn.datasets.synth import as_model_input
    from paig_reproduction_amd.nn.network.physics_models import PhysicsNet
    from render_pool import render_distinct
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = PhysicsNet(task, 100, 1, cell, seq_len, ins, pred, 3.0, False, True, size * size, "conv_encoder",
                   "conv_st_decoder", device=dev).to(dev)
    m.conv_math = "split"
    # B distinct sequences (no tiling: an error aliasing sequence i with
    # i + n would be invisible in a tiled batch)
    x = torch.from_numpy(as_model_input(render_distinct(task, B, seq_len, seed)))
    state = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    cfg = O.Cfg(task, cell, seq_len, ins, pred, size, 3.0)
    return m, x, state, cfg


def _hip_step(m, x):
    dev = torch.device("cuda:0")
    xd = x.to(dev)
    m.output = m(xd)
    loss, (pred, extrap, recons) = m.compute_loss()
    m.zero_grad(set_to_none=True)
    loss.backward()
    torch.cuda.synchronize()
    out = {"enc_pos": m.enc_pos, "enc_masks": m.enc_masks, "recons_out": m.recons_out, "output_seq": m.output,
           "pos_vel_seq": m.pos_vel_seq}
    out = {k: v.detach().double().cpu().numpy() for k, v in out.items()}
    L = {"train": float(loss.detach()), "extrap": float(extrap.detach()), "recons": float(recons.detach())}
    g = {k: p.grad.detach().double().cpu().numpy() for k, p in m.named_parameters() if p.grad is not None}
    sse = (m._sse_rec.detach().double().cpu().numpy(), m._sse_roll.detach().double().cpu().numpy())
    return out, L, g, sse


# the rollout-derived quantities (pos_vel_seq split into positions and
# velocities, each against its own scale: VERDICT r05 weak 1d)
ROLLOUT_KEYS = ("output_seq", "pos_vel_seq", "pos_vel_seq.pos", "pos_vel_seq.vel", "loss_extrap", "loss_train")


def _rollout_parts(out, L):
    """float64 numpy views of the rollout-derived outputs and losses."""
    f = lambda t: t.detach().double().numpy() if torch.is_tensor(t) else np.asarray(t, dtype=np.float64)  # noqa: E731
    pv = f(out["pos_vel_seq"])
    D = pv.shape[-1] // 2
    return {"output_seq": f(out["output_seq"]).reshape(-1), "pos_vel_seq": pv.reshape(-1),
            "pos_vel_seq.pos": pv[..., :D], "pos_vel_seq.vel": pv[..., D:],
            "loss_extrap": np.float64(float(L["extrap"])), "loss_train": np.float64(float(L["train"]))}


def _full_check(tag, task, cell, seq_len, ins, pred, size, B, rollout_rtol=RTOL, seed=3, ensemble=ENSEMBLE_FULL,
                vel_rtol=RTOL):
    """Whole-batch outputs / losses vs the fp32 oracle and every gradient
    element vs the float64 oracle within the fp32 envelope."""
    import time
    _threads()
    t0 = time.time()
    m, x, state, cfg = _model(task, cell, seq_len, ins, pred, size, B, seed=seed)
    out, L, g, _ = _hip_step(m, x)
    del m
    torch.cuda.empty_cache()
    o32, L32, g32 = O.train_step(state, cfg, x)
    errs = {}
    for k in OUT_KEYS:
        errs[k] = rel_err(out[k].reshape(-1), o32[k].detach().double().numpy().reshape(-1))
    hip_r = _rollout_parts(out, L)
    r32 = _rollout_parts(o32, L32)
    errs.update({k: rel_err(hip_r[k], r32[k]) for k in ("pos_vel_seq.pos", "pos_vel_seq.vel")})
    for k in ("train", "extrap", "recons"):
        errs["loss_" + k] = rel_err(np.float64(L[k]), np.float64(float(L32[k].detach())))
    del o32, L32
    print(tag, "outputs/losses vs fp32 oracle:", {k: f"{v:.2e}" for k, v in errs.items()})
    # everything the rollout does not amplify: 1e-4 (north star) against fp32
    over = {k: v for k, v in errs.items() if k not in ROLLOUT_KEYS and v > RTOL}
    assert not over, over
    # the rollout-derived outputs against the float64 oracle: bar = the fixed
    # bar or ENVELOPE_K x the fp32 spread, whichever is larger.  The rollout
    # amplifies last-bit differences: 3bp's gravity is chaotic, and a
    # bouncing ball one ulp from a wall bounces one substep earlier or later
    # in a distinct sequence, so honest fp32 runs (the oracle on one-ulp-
    # perturbed weights) differ from float64 by more than 1e-4 there.
    o64, L64, g64 = O.train_step_f64(state, cfg, x)
    r64 = _rollout_parts(o64, L64)
    del o64
    g64 = {k: v.detach().double().numpy() for k, v in g64.items()}
    assert sorted(g) == sorted(g64), set(g) ^ set(g64)
    ospread = {k: rel_err(r32[k], r64[k]) for k in r64}
    spread = {k: rel_err(g32[k].detach().double().numpy(), g64[k]) for k in g64}
    del g32, r32
    for s_ in range(ensemble):
        op, Lp, gp = O.train_step(_ulp_perturbed(state, s_), cfg, x)
        rp = _rollout_parts(op, Lp)
        del op
        for k in r64:
            ospread[k] = max(ospread[k], rel_err(rp[k], r64[k]))
        for k in g64:
            spread[k] = max(spread[k], rel_err(gp[k].detach().double().numpy(), g64[k]))
        del gp, rp
    fixed = {k: vel_rtol if k == "pos_vel_seq.vel" else rollout_rtol for k in r64}
    orow = {k: (rel_err(hip_r[k], r64[k]), ospread[k], max(fixed[k], ENVELOPE_K * ospread[k])) for k in r64}
    print(tag, "rollout outputs vs float64 (hip, fp32 spread, bar):",
          {k: tuple(f"{u:.2e}" for u in v) for k, v in orow.items()})
    bad = {k: v for k, v in orow.items() if v[0] > v[2]}
    assert not bad, bad
    rows = {k: (rel_err(g[k], g64[k]), spread[k], max(ENVELOPE_K * spread[k], ENVELOPE_FLOOR)) for k in g64}
    worst = max(rows.items(), key=lambda kv: kv[1][0] / kv[1][2])
    print(tag, "worst gradient (hip, fp32 spread, bar):", worst, f"({time.time() - t0:.0f} s)")
    bad = {k: v for k, v in rows.items() if v[0] > v[2]}
    assert not bad, bad
    return errs, rows


# (the oracle's CPU steps dominate: mnist B=256 is ~21 s per fp32 / float64
# step on the GPU box's 16 cores, so its test gets a longer limit rather than
# a smaller envelope ensemble)
@pytest.mark.timeout(300)
def test_config1_spring_b100_seq50_matches_oracle():
    _full_check("config #1", "spring_color", "spring_ode_cell", 50, 4, 6, 32, 100)


@pytest.mark.timeout(300)
def test_config3_3bp_b512_matches_oracle():
    _full_check("config #3", "3bp_color", "gravity_ode_cell", 20, 4, 12, 36, 512, ROLLOUT_RTOL_3BP, seed=5,
                vel_rtol=VEL_RTOL_3BP)


@pytest.mark.timeout(600)
def test_config4_mnist_b256_matches_oracle():
    _full_check("config #4", "mnist_spring_color", "spring_ode_cell", 12, 3, 7, 64, 256, seed=5)


@pytest.mark.timeout(300)
def test_config5_bouncing_b1024_r96_matches_oracle():
    _full_check("config #5", "bouncing_balls", "bouncing_ode_cell", 100, 4, 6, 32, 1024, seed=5)


@pytest.mark.timeout(600)
def test_config2_spring_bf16_b512_matches_bf16_oracle():
    """Config #2 (spring_color bf16, B=512, seq 50) on the whole batch of
    distinct sequences against the oracle in the same bf16-operand
    arithmetic, within the bf16 envelope (tests/test_gpu_parity.py
    bf16_envelope_check).  Weights: the fixtures' live-layer scaling
    (tests/golden/weights.py), so every layer's bf16 rounding matters (at the
    default initialisation the masks come out nearly uniform)."""
    import time
    from test_gpu_parity import bf16_envelope_check
    from weights import golden_state
    _threads()
    t0 = time.time()
    m, x, _, cfg = _model("spring_color", "spring_ode_cell", 50, 4, 6, 32, 512, seed=7)
    sd = m.state_dict()
    gs = golden_state({k: (tuple(v.shape), str(v.cpu().numpy().dtype)) for k, v in sd.items()}, 3)
    m.load_state_dict({k: torch.from_numpy(v).to("cuda:0") for k, v in gs.items()})
    state = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    m.conv_math = "bf16"
    m.output = m(x.to("cuda:0"))
    train_loss, (pred, extrap, recons) = m.compute_loss()
    m.zero_grad(set_to_none=True)
    train_loss.backward()
    torch.cuda.synchronize()
    bf16_envelope_check(m, x, state, cfg, train_loss, extrap, recons, "config #2", ensemble=5)
    print(f"config #2: {time.time() - t0:.0f} s")
