"""fp32 honesty of the HIP step: for every golden config, each output and
each parameter gradient of the HIP step (split and fp32 conv arithmetic) must
sit within ENVELOPE_K times the fp32 reference's own distance to a float64
run of the same step (tests/envelope.py).  This is what makes the "fp32"
label of the split-precision path (f16 hi/lo pieces on the 16-bit matrix
cores) a measured claim rather than an output-only one.  The measured table
is kept in profiles/r02_grad_envelope.json (tools/grad_envelope.py)."""
import pytest
import torch

from helpers import GOLDEN
from envelope import envelope, ENVELOPE_K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("conv_math", ["split", "fp32"])
@pytest.mark.parametrize("name", GOLDEN)
def test_within_fp32_envelope(name, conv_math):
    rows = envelope(name, conv_math, torch.device("cuda:0"))
    over = {k: f"hip {a:.2e} > {ENVELOPE_K:g} x fp32 {b:.2e}" for k, (a, b, c) in rows.items() if a > c}
    worst = max(rows.items(), key=lambda kv: kv[1][0] / kv[1][2])
    print(name, conv_math, "worst hip/bar:", worst[0], f"{worst[1][0]:.2e}/{worst[1][2]:.2e}")
    assert not over, over
