"""The whole U-Net through the C ABI alone (paig_unet_workspace / _fwd / _bwd,
csrc/unet.hip) against the Python engine's U-Net stages
(model.encoder.shallow_unet / .unet, nn/network/native_modules.py, which the
module tests check against the oracle): the composite runs the same kernels
in the same order, so logits and every conv's weight and bias gradient must
be BIT-IDENTICAL.  Reference: ShallowUNet blocks.py:240-308, UNet :106-237.
"""
import ctypes

import pytest
import torch

from helpers import load_golden
from oracle import physics_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
MATH = {"split": 128, "bf16": 256, "fp32": 0}


def _parr(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


@pytest.mark.parametrize("name,which,math,N", [("spring_s12", "shallow_unet", "split", 7),
                                               ("spring_s12", "shallow_unet", "bf16", 5),
                                               ("3bp_s20", "shallow_unet", "split", 6),
                                               ("mnist_s12", "unet", "split", 3)])
def test_unet_abi_matches_engine(name, which, math, N):
    from paig_reproduction_amd._lib import lib
    from test_gpu_parity import _model
    L = lib()
    z = load_golden(name)
    cfg, _ = O.cfg_from_golden(z)
    m = _model(z, DEV)
    m.conv_math = math
    H, K = cfg.size, cfg.n_objs
    torch.manual_seed(0)
    x = torch.rand(N, 3, H, H, device=DEV)
    # the engine's path: logits, then the gradients of sum(logits * R)
    mod = getattr(m.encoder, which)
    logits = mod(x)
    R = torch.randn_like(logits)
    m.zero_grad(set_to_none=True)
    (logits * R).sum().backward()
    torch.cuda.synchronize()
    pd = dict(m.named_parameters())
    prefix = "encoder." + which + "."
    nconv = 13 if which == "shallow_unet" else 18
    ws_ = [pd[f"{prefix}c{i + 1}.weight"].detach() for i in range(nconv)]
    bs_ = [pd[f"{prefix}c{i + 1}.bias"].detach() for i in range(nconv)]
    # the C ABI alone
    net = 0 if which == "shallow_unet" else 1
    nbytes = int(L.paig_unet_workspace(net, N, H, K, MATH[math]))
    assert nbytes > 0
    ws = torch.empty(nbytes // 4 + 1, device=DEV)
    lg = torch.empty(N, K, H, H, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    L.paig_unet_fwd(net, N, H, K, MATH[math], x.data_ptr(), 3 * H * H, 0, 0, _parr([t.data_ptr() for t in ws_]),
                    _parr([t.data_ptr() for t in bs_]), lg.data_ptr(), ws.data_ptr(), nbytes, st)
    torch.cuda.synchronize()
    assert torch.equal(lg, logits.detach()), f"logits differ: {(lg - logits).abs().max().item():.3e}"
    dwb = [torch.full((w.numel() + w.shape[0],), float("nan"), device=DEV) for w in ws_]
    L.paig_unet_bwd(net, N, H, K, MATH[math], x.data_ptr(), 3 * H * H, 0, 0, _parr([t.data_ptr() for t in ws_]),
                    lg.data_ptr(), R.contiguous().data_ptr(), _parr([t.data_ptr() for t in dwb]), ws.data_ptr(),
                    nbytes, st)
    torch.cuda.synchronize()
    for i in range(nconv):
        gw, gb = pd[f"{prefix}c{i + 1}.weight"].grad, pd[f"{prefix}c{i + 1}.bias"].grad
        nw = gw.numel()
        assert torch.equal(dwb[i][:nw], gw.reshape(-1)), f"c{i + 1}.weight"
        assert torch.equal(dwb[i][nw:], gb.reshape(-1)), f"c{i + 1}.bias"


def test_unet_abi_rejects_bad_arguments():
    from paig_reproduction_amd._lib import lib, PaigError
    L = lib()
    assert L.paig_unet_workspace(2, 4, 32, 2, 128) == 0   # no such net
    assert L.paig_unet_workspace(0, 4, 32, 2, 64) == 0    # no such conv math
    x = torch.zeros(4, 3, 32, 32, device=DEV)
    with pytest.raises(PaigError):   # workspace too small
        L.paig_unet_fwd(0, 4, 32, 2, 128, x.data_ptr(), 3 * 1024, 0, 0, _parr([0] * 13), _parr([0] * 13),
                        x.data_ptr(), x.data_ptr(), 16, torch.cuda.current_stream().cuda_stream)
