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


@pytest.mark.parametrize("alt", [16, 32])
@pytest.mark.parametrize("N", [3, 40])
def test_unet_upsample_backward_in_dgrad_epilogue_is_bit_identical(N, alt):
    """alt 16: the UNet's c9 / c12 / c15 data gradients with the upsample's
    backward in their epilogue (paig_conv2d_fwd_pw flags & 512, the default)
    against the same dgrads followed by paig_upsample2_bwd
    (PAIG_UNET_STANDALONE_UP); alt 32: c4's separate weight and data
    gradients with pool2's backward folded into their dY staging
    (paig_conv2d_wgrad_pf, the dgrad's flags 8 | 64) against
    paig_maxpool2_bwd_relu then the plain kernels (PAIG_UNET_STANDALONE_POOL).
    Every conv's weight and bias gradient bit-identical.  Reference:
    blocks.py:186-197 (pools), 206,219,229 (upsamples)."""
    from paig_reproduction_amd._lib import lib
    L = lib()
    H, K, net, nconv, math = 64, 2, 1, 18, 128
    torch.manual_seed(7)
    ws_ = [None] * nconv
    chans = [(3, 16, 3), (16, 16, 3), (16, 32, 3), (32, 32, 3), (32, 64, 3), (64, 64, 3), (64, 128, 3), (128, 128, 3),
             (128, 32, 3), (96, 64, 3), (64, 64, 3), (64, 32, 3), (64, 32, 3), (32, 32, 3), (32, 32, 3), (48, 16, 3),
             (16, 16, 3), (16, K, 1)]
    ws_ = [torch.randn(co, ci, k, k, device=DEV) * (2.0 / (ci * k * k)) ** 0.5 for ci, co, k in chans]
    bs_ = [torch.randn(co, device=DEV) * 0.1 for _, co, _ in chans]
    x = torch.rand(N, 3, H, H, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for flags in (0, alt):
        nbytes = int(L.paig_unet_workspace_ex(net, N, H, K, math, flags))
        ws = torch.empty(nbytes // 4 + 1, device=DEV)
        lg = torch.empty(N, K, H, H, device=DEV)
        L.paig_unet_fwd_ex(net, N, H, K, math, flags, x.data_ptr(), 3 * H * H, 0, 0,
                           _parr([t.data_ptr() for t in ws_]), _parr([t.data_ptr() for t in bs_]), lg.data_ptr(), None,
                           None, ws.data_ptr(), nbytes, None, None, st)
        torch.manual_seed(11)
        R = torch.randn(N, K, H, H, device=DEV)
        dwb = [torch.full((w.numel() + w.shape[0],), float("nan"), device=DEV) for w in ws_]
        L.paig_unet_bwd_ex(net, N, H, K, math, flags, x.data_ptr(), 3 * H * H, 0, 0,
                           _parr([t.data_ptr() for t in ws_]), lg.data_ptr(), R.data_ptr(),
                           _parr([t.data_ptr() for t in dwb]), 0, None, None, None, None, None, ws.data_ptr(), nbytes,
                           None, None, st)
        torch.cuda.synchronize()
        out[flags] = (lg.clone(), dwb)
    assert torch.equal(out[0][0], out[alt][0])
    for i in range(nconv):
        a, b = out[0][1][i], out[alt][1][i]
        assert torch.isfinite(a).all(), f"c{i + 1}"
        assert torch.equal(a, b), f"c{i + 1}: max |d| {(a - b).abs().max().item():.3e}"


@pytest.mark.parametrize("cin,cout,H", [(128, 32, 16), (64, 32, 32), (32, 32, 64)])
@pytest.mark.parametrize("F", [5, 700])
def test_dgrad_upsample_epilogue_kernel(cin, cout, H, F):
    """paig_conv2d_fwd_pw flags & 512 (dgrad of a conv whose input was the 2x
    upsample, writing the upsample source's gradient with its ReLU' mask)
    bit-identical to the dgrad then paig_upsample2_bwd; F = 700 gives every
    persistent block several frames (the carried rows)."""
    from paig_reproduction_amd._lib import lib
    L = lib()
    torch.manual_seed(cin + H + F)
    hs = H // 2
    dy = torch.randn(F, cout, H, H, device=DEV)
    w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    src = torch.randn(F, cin, hs, hs, device=DEV)   # the upsample source (ReLU output: mask src > 0)
    st = torch.cuda.current_stream().cuda_stream
    full = torch.empty(F, cin, H, H, device=DEV)
    rc = L.paig_conv2d_fwd_pw(dy.data_ptr(), cout * H * H, 0, 0, full.data_ptr(), cin * H * H, None, 0, w.data_ptr(),
                              None, F, cout, cin, H, H, 3, 8 | 128, None, 0, None, 0, None, st)
    assert rc == 0
    ref = torch.empty(F, cin, hs, hs, device=DEV)
    L.paig_upsample2_bwd(full.data_ptr(), cin * H * H, src.data_ptr(), cin * hs * hs, ref.data_ptr(), cin * hs * hs, F,
                         cin, hs, hs, H, H, 1, st)
    got = torch.full((F, cin, hs, hs), float("nan"), device=DEV)
    assert L.paig_conv2d_mfma_supported(0, cout, cin, H, H, 3, 8 | 128 | 512) == 1
    rc = L.paig_conv2d_fwd_pw(dy.data_ptr(), cout * H * H, 0, 0, got.data_ptr(), cin * hs * hs, src.data_ptr(),
                              cin * hs * hs, w.data_ptr(), None, F, cout, cin, H, H, 3, 8 | 128 | 512 | 2, None, 0,
                              None, 0, None, st)
    assert rc == 0
    torch.cuda.synchronize()
    assert torch.equal(got, ref), f"max |d| {(got - ref).abs().max().item():.3e}"
