"""Per-parameter gradient errors of the HIP step vs a golden fixture, for
each conv arithmetic (diagnostic; run on the GPU box from the repo root):
    python tools/grad_errs.py mnist_s12 split fp32"""
import os
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]
import torch  # noqa: E402
from helpers import load_golden, grad_checks  # noqa: E402
from test_gpu_parity import _model, _input  # noqa: E402


def main():
    name = sys.argv[1]
    z = load_golden(name)
    dev = torch.device("cuda:0")
    for cm in sys.argv[2:]:
        m = _model(z, dev)
        m.conv_math = cm
        m.output = m(_input(z, dev))
        loss, _ = m.compute_loss()
        m.zero_grad(set_to_none=True)
        loss.backward()
        torch.cuda.synchronize()
        grads = {k: p.grad for k, p in m.named_parameters() if p.grad is not None}
        errs = grad_checks(z, grads, 1e9)
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:12]
        print(cm, " ".join(f"{k}={v:.2e}" for k, v in worst), flush=True)


if __name__ == "__main__":
    main()
