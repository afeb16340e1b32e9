"""Pin the CPU oracle (oracle/physics_oracle.py) to the reference's own outputs.

The golden vectors were produced by running the reference itself
(tests/golden/gen_golden.py); the oracle is an independent restatement.
Both run on CPU fp32 with the same aten ops, so the bar here is tighter
than the HIP parity bar.
"""
import pytest
import torch

from helpers import GOLDEN, load_golden, golden_weights, assert_close, grad_checks
from oracle import physics_oracle as O

# Same aten ops on the same CPU: outputs agree to ~1e-7 except where the
# rollout amplifies last-bit differences of op ordering (3bp gravity is chaotic:
# 1.7e-5 on its frames).
ORACLE_RTOL = 2e-6
ROLLOUT_RTOL = {"3bp_s20": 5e-5}


@pytest.mark.parametrize("name", GOLDEN)
def test_oracle_matches_reference(name):
    torch.set_num_threads(4)
    z = load_golden(name)
    cfg, B = O.cfg_from_golden(z)
    state = golden_weights(z)
    x = O.input_from_u8(z["input_u8"])
    out, L, grads = O.train_step(state, cfg, x)
    for k in ("enc_pos", "enc_masks", "recons_out"):
        assert_close(out[k], z[k], ORACLE_RTOL, k)
    for k in ("output_seq", "pos_vel_seq"):
        assert_close(out[k], z[k], ROLLOUT_RTOL.get(name, 1e-5), k)
    assert_close(L["recons"], z["loss_recons"], ORACLE_RTOL, "recons")
    assert_close(L["extrap"], z["loss_extrap"], ORACLE_RTOL, "extrap")
    assert_close(L["pred"], z["loss_pred_true"], ORACLE_RTOL, "pred")
    assert_close(L["train"], z["loss_train"], ORACLE_RTOL, "train")
    grad_checks(z, grads, ROLLOUT_RTOL.get(name, 2e-5))
    # the oracle's live-parameter set is exactly the set the reference grads
    assert sorted(grads) == sorted(str(k) for k in z["grad_keys"])
