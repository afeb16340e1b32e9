"""The fused layer backward (csrc/conv_bwd.hip, paig_conv2d_bwd): a U-Net
conv's data gradient AND weight + bias gradients in one launch, vs float64
torch conv2d backward (the aten convolution_backward the reference's
ShallowUNet runs, nn/network/blocks.py:246-276), on every fused shape of the
ShallowUNet at 32 x 32 (spring, bouncing) and 36 x 36 (3bp), in split (f16
hi/lo, fp32-accurate) and bf16 arithmetic.  Cases: ragged frame counts,
ReLU' mask + accumulation into an existing gradient, weight images from
paig_conv_wprep (bit-identical to in-kernel staging), activations and
gradients spread over many binades (the running dY exponent rescales the
accumulators), and agreement with the separate dgrad / wgrad kernels."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from helpers import rel_err

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
XMAX_SLOTS = 2048
TOL = {128: 1e-5, 256: 8e-3}
SHAPES = [(8, 8, 32), (8, 16, 16), (16, 16, 16), (16, 32, 8), (32, 32, 8), (32, 16, 16), (24, 8, 32),
          (16, 16, 64), (16, 32, 32),
          (8, 8, 36), (8, 16, 18), (16, 16, 18), (32, 16, 18), (24, 8, 36)]


def L():
    from paig_reproduction_amd._lib import lib
    return lib()


def st():
    return torch.cuda.current_stream().cuda_stream


def p(t):
    return None if t is None else t.data_ptr()


def _wprep(w, cin, cout):
    n = int(L().paig_conv_wprep_size(cout, cin, 3))
    buf = torch.empty(n, dtype=torch.int16, device=DEV)
    L().paig_conv_wprep(1, (ctypes.c_void_p * 1)(p(w)), (ctypes.c_int * 1)(cout), (ctypes.c_int * 1)(cin),
                        (ctypes.c_int * 1)(3), (ctypes.c_int * 1)(1), (ctypes.c_void_p * 1)(p(buf)), st())
    return buf


def _fused(x, w, dy, dx0, aux, mode, xmax, wprep=None, nmax=512):
    F_, cin, hw = x.shape[0], x.shape[1], x.shape[2]
    cout = w.shape[0]
    dx = dx0.clone()
    flags = mode | (4 if dx0.abs().sum() > 0 else 0) | (2 if aux is not None else 0)
    slab = torch.empty(nmax * (cout * cin * 9 + cout), device=DEV)
    nb = ctypes.c_int(0)
    L().paig_conv2d_bwd(p(x), cin * hw * hw, 0, 0, p(dy), cout * hw * hw, p(dx), cin * hw * hw, p(aux),
                        cin * hw * hw, p(w), p(slab), nmax, ctypes.byref(nb), F_, cin, cout, hw, hw, 3, flags,
                        p(xmax), XMAX_SLOTS if xmax is not None else 0, None, 0, None, 0, p(wprep), st())
    g = torch.empty(cout * cin * 9 + cout, device=DEV)
    L().paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st())
    torch.cuda.synchronize()
    n = cout * cin * 9
    return dx, g[:n].view_as(w), g[n:]


def _xmax_of(x, w, b, mode):
    """The forward of x, recording its per-block max |x| slots (what the
    training step hands the backward)."""
    F_, cin, hw = x.shape[0], x.shape[1], x.shape[2]
    cout = w.shape[0]
    xmax = torch.zeros(XMAX_SLOTS, device=DEV)
    out = torch.empty(F_, cout, hw, hw, device=DEV)
    L().paig_conv2d_fwd_ex(p(x), cin * hw * hw, 0, 0, p(out), cout * hw * hw, None, 0, p(w), p(b), F_, cin, cout,
                           hw, hw, 3, mode, p(xmax), XMAX_SLOTS, st())
    return xmax


def _ref(x, w, dy, dx0, aux):
    xr = x.double().cpu().requires_grad_(True)
    wr = w.double().cpu().requires_grad_(True)
    y = F.conv2d(xr, wr, padding="same")
    y.backward(dy.double().cpu())
    dx = xr.grad + dx0.double().cpu()
    if aux is not None:
        dx = dx * (aux.cpu() > 0)
    return dx, wr.grad, dy.double().cpu().sum((0, 2, 3))


@pytest.mark.parametrize("mode", [128, 256])
@pytest.mark.parametrize("cin,cout,hw", SHAPES)
def test_fused_backward_matches_fp64(cin, cout, hw, mode):
    assert L().paig_conv2d_bwd_supported(cin, cout, hw, hw, 3, mode) == 1
    tol = TOL[mode]
    # nmax 2: two persistent blocks walk every tile
    for F_, relu_acc, nmax in ((5, True, 512), (3, False, 512), (1, True, 512), (5, True, 2)):
        torch.manual_seed(cin * 1000 + cout * 10 + hw + F_)
        x = torch.relu(torch.randn(F_, cin, hw, hw, device=DEV))
        w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.2
        b = torch.randn(cout, device=DEV)
        dy = torch.randn(F_, cout, hw, hw, device=DEV)
        dx0 = torch.full((F_, cin, hw, hw), 0.5, device=DEV) if relu_acc else torch.zeros(F_, cin, hw, hw, device=DEV)
        aux = x if relu_acc else None
        xmax = _xmax_of(x, w, b, mode) if mode == 128 else None
        dx, gw, gb = _fused(x, w, dy, dx0, aux, mode, xmax, nmax=nmax)
        rdx, rgw, rgb = _ref(x, w, dy, dx0, aux)
        assert rel_err(dx, rdx) <= tol, ("dx", F_)
        assert rel_err(gw, rgw) <= tol, ("dw", F_)
        assert rel_err(gb, rgb) <= 1e-5, ("db", F_)


@pytest.mark.parametrize("cin,cout,hw", [(8, 8, 32), (32, 32, 8), (24, 8, 32), (16, 16, 18), (32, 16, 18)])
def test_fused_backward_wprep_bit_identical(cin, cout, hw):
    """Weight images from paig_conv_wprep (once per step) give bit-identical
    results to the kernel's own staging."""
    torch.manual_seed(cin + cout + hw)
    F_ = 4
    x = torch.relu(torch.randn(F_, cin, hw, hw, device=DEV))
    w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.2
    b = torch.randn(cout, device=DEV)
    dy = torch.randn(F_, cout, hw, hw, device=DEV)
    dx0 = torch.full((F_, cin, hw, hw), 0.25, device=DEV)
    xmax = _xmax_of(x, w, b, 128)
    a = _fused(x, w, dy, dx0, x, 128, xmax)
    c = _fused(x, w, dy, dx0, x, 128, xmax, _wprep(w, cin, cout))
    for u, v in zip(a, c):
        assert torch.equal(u, v)


@pytest.mark.parametrize("act_scale,dy_scale", [(40.0, 1.0), (1e-5, 1e-12), (1.0, 1e9), (3e4, 1e6)])
def test_fused_backward_any_range(act_scale, dy_scale):
    """Gradients whose frames differ by 12 binades (the running exponent
    lowers mid-launch and rescales the accumulators) and activations at any
    magnitude keep fp32 accuracy (float64 reference)."""
    cin, cout, hw, F_ = 16, 16, 16, 9
    torch.manual_seed(11)
    x = torch.relu(torch.randn(F_, cin, hw, hw, device=DEV)) * act_scale
    w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.2
    b = torch.randn(cout, device=DEV)
    dy = torch.randn(F_, cout, hw, hw, device=DEV) * dy_scale
    dy *= torch.logspace(-6, 6, F_, device=DEV).view(F_, 1, 1, 1)
    xmax = _xmax_of(x, w, b, 128)
    dx, gw, gb = _fused(x, w, dy, torch.zeros_like(x), x, 128, xmax)
    rdx, rgw, rgb = _ref(x, w, dy, torch.zeros_like(x), x)
    # dX per frame (each frame's own magnitude)
    for f in range(F_):
        assert rel_err(dx[f], rdx[f]) <= 1e-5, f
    assert rel_err(gw, rgw) <= 1e-5
    assert rel_err(gb, rgb) <= 1e-5


@pytest.mark.parametrize("cin,cout,hw", [(8, 8, 32), (24, 8, 32), (32, 16, 16)])
def test_fused_backward_matches_separate_kernels(cin, cout, hw):
    """The fused launch and the separate dgrad / wgrad kernels agree (both
    fp32-accurate; different k order and scales: within 2e-6)."""
    torch.manual_seed(7)
    F_ = 6
    x = torch.relu(torch.randn(F_, cin, hw, hw, device=DEV))
    w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.2
    b = torch.randn(cout, device=DEV)
    dy = torch.randn(F_, cout, hw, hw, device=DEV)
    xmax = _xmax_of(x, w, b, 128)
    dx, gw, gb = _fused(x, w, dy, torch.zeros_like(x), x, 128, xmax)
    dx2 = torch.empty_like(x)
    L().paig_conv2d_fwd(p(dy), cout * hw * hw, 0, 0, p(dx2), cin * hw * hw, p(x), cin * hw * hw, p(w), None, F_, cout,
                        cin, hw, hw, 3, 8 | 2 | 128, st())
    nmax = 256
    slab = torch.empty(nmax * (cout * cin * 9 + cout), device=DEV)
    nb = ctypes.c_int(0)
    L().paig_conv2d_wgrad_ex(p(x), cin * hw * hw, 0, 0, p(dy), cout * hw * hw, p(slab), nmax, ctypes.byref(nb), F_, cin,
                             cout, hw, hw, 3, 128, p(xmax), XMAX_SLOTS, st())
    g = torch.empty(cout * cin * 9 + cout, device=DEV)
    L().paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st())
    torch.cuda.synchronize()
    n = cout * cin * 9
    assert rel_err(dx, dx2) <= 2e-6
    assert rel_err(gw, g[:n].view_as(w)) <= 2e-6
    assert rel_err(gb, g[n:]) <= 2e-6


@pytest.mark.parametrize("mode", [128, 256])
@pytest.mark.parametrize("cin,cout,hw", [(32, 16, 16), (16, 16, 32), (16, 16, 36), (32, 16, 18)])
def test_fused_backward_upsample_input(cin, cout, hw, mode):
    """c7 / c10 (blocks.py:289-290,298-299): the conv input is the 2x bilinear
    upsample (torchvision Resize) of a ReLU'd half-resolution source.  One
    launch gives the weight / bias gradients and the SOURCE's gradient (the
    upsample's backward folded in, ReLU' of the source applied); float64
    autograd through F.interpolate + conv2d is the reference."""
    assert L().paig_conv2d_bwd_supported(cin, cout, hw, hw, 3, mode | 32) == 1
    tol = TOL[mode]
    # nmax 2: two persistent blocks walk every tile (the staging of a block's
    # later tiles must not see what its earlier tiles left in the LDS)
    for F_, nmax in ((3, 512), (1, 512), (3, 2)):
        torch.manual_seed(cin + cout + hw + F_)
        xs = torch.relu(torch.randn(F_, cin, hw // 2, hw // 2, device=DEV))
        w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.2
        b = torch.randn(cout, device=DEV)
        dy = torch.randn(F_, cout, hw, hw, device=DEV)
        xr = xs.double().cpu().requires_grad_(True)
        wr = w.double().cpu().requires_grad_(True)
        xu = F.interpolate(xr, size=(hw, hw), mode="bilinear", align_corners=False, antialias=True)
        F.conv2d(xu, wr, padding="same").backward(dy.double().cpu())
        rdx = xr.grad * (xs.cpu() > 0)
        hs = hw // 2
        xmax = None
        if mode == 128:
            xmax = torch.zeros(XMAX_SLOTS, device=DEV)
            out = torch.empty(F_, cout, hw, hw, device=DEV)
            L().paig_conv2d_fwd_ex(p(xs), cin * hs * hs, 0, 0, p(out), cout * hw * hw, None, 0, p(w), p(b), F_, cin,
                                   cout, hw, hw, 3, 32 | mode, p(xmax), XMAX_SLOTS, st())
        dx = torch.full((F_, cin, hs, hs), float("nan"), device=DEV)   # write mode: every element written
        slab = torch.empty(nmax * (cout * cin * 9 + cout), device=DEV)
        nb = ctypes.c_int(0)
        L().paig_conv2d_bwd(p(xs), cin * hs * hs, 0, 0, p(dy), cout * hw * hw, p(dx), cin * hs * hs, p(xs),
                            cin * hs * hs, p(w), p(slab), nmax, ctypes.byref(nb), F_, cin, cout, hw, hw, 3,
                            mode | 32 | 2, p(xmax), XMAX_SLOTS if xmax is not None else 0, None, 0, None, 0, None,
                            st())
        g = torch.empty(cout * cin * 9 + cout, device=DEV)
        L().paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st())
        torch.cuda.synchronize()
        n = cout * cin * 9
        assert torch.isfinite(dx).all()
        assert rel_err(dx, rdx) <= tol, ("dx", F_)
        assert rel_err(g[:n].view_as(w), wr.grad) <= tol, ("dw", F_)
        assert rel_err(g[n:], dy.double().cpu().sum((0, 2, 3))) <= 1e-5, ("db", F_)


@pytest.mark.parametrize("mode", [128, 256])
@pytest.mark.parametrize("cin,cout,hw", [(8, 8, 32), (16, 16, 16), (16, 16, 64), (8, 8, 36), (16, 16, 18)])
def test_fused_backward_pool_fold(cin, cout, hw, mode):
    """c2 / c4 (blocks.py:249-250, 253-254): the layer's ReLU'd output feeds
    the skip concat AND a 2x2 max pool.  The forward's fused pool writes one
    code byte per window (ReLU' bits + argmax, paig_conv2d_fwd_pwc); the
    layer backward folds the pool's backward into its dY staging
    (dY = ReLU'(y) (dY_skip + scatter_argmax(d pooled))).  Reference: float64
    autograd through conv2d + relu + max_pool2d."""
    assert L().paig_conv2d_bwd_supported(cin, cout, hw, hw, 3, mode | 64) == 1
    tol = TOL[mode]
    hp = hw // 2
    for F_, nmax in ((4, 512), (1, 512), (4, 2)):   # nmax 2: blocks walk many tiles
        torch.manual_seed(cin + cout + hw + F_ + mode)
        x = torch.relu(torch.randn(F_, cin, hw, hw, device=DEV))
        w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.2
        b = torch.randn(cout, device=DEV) * 0.1
        gy = torch.randn(F_, cout, hw, hw, device=DEV)     # the skip path's gradient (c11's dgrad)
        gp = torch.randn(F_, cout, hp, hp, device=DEV)     # the pooled output's gradient (c3's dgrad)
        # GPU forward: conv + ReLU + fused pool with window codes (+ the X maxima)
        y = torch.empty(F_, cout, hw, hw, device=DEV)
        pool = torch.empty(F_, cout, hp, hp, device=DEV)
        cfs = -(-cout // 8) * 8 * hp * hp
        code = torch.empty(F_ * cfs, dtype=torch.uint8, device=DEV)
        xmax = torch.zeros(XMAX_SLOTS, device=DEV)
        if L().paig_conv2d_mfma_supported(0, cin, cout, hw, hw, 3, mode | 64):
            L().paig_conv2d_fwd_pwc(p(x), cin * hw * hw, 0, 0, p(y), cout * hw * hw, None, 0, p(w), p(b), F_, cin,
                                    cout, hw, hw, 3, 1 | 64 | mode, p(xmax) if mode == 128 else None,
                                    XMAX_SLOTS if mode == 128 else 0, p(pool), cout * hp * hp, p(code), cfs, None, st())
        else:
            # 3bp's 36 / 18: the conv cannot pool in its epilogue; the
            # standalone pool writes the same codes (paig_maxpool2_fwd_codes)
            L().paig_conv2d_fwd_pwc(p(x), cin * hw * hw, 0, 0, p(y), cout * hw * hw, None, 0, p(w), p(b), F_, cin,
                                    cout, hw, hw, 3, 1 | mode, p(xmax) if mode == 128 else None,
                                    XMAX_SLOTS if mode == 128 else 0, None, 0, None, 0, None, st())
            assert L().paig_maxpool2_fwd_codes(p(y), cout * hw * hw, p(pool), cout * hp * hp, p(code), cfs, F_, cout,
                                               hw, hw, st()) == 0
            ref = torch.empty_like(pool)
            L().paig_maxpool2_fwd(p(y), cout * hw * hw, p(ref), cout * hp * hp, F_, cout, hw, hw, st())
            torch.cuda.synchronize()
            assert torch.equal(pool, ref)   # bit-identical pooled values
        torch.cuda.synchronize()
        xd, wd = x.double().cpu(), w.double().cpu()
        assert rel_err(pool, F.max_pool2d(torch.relu(F.conv2d(xd, wd, b.double().cpu(), padding="same")), 2)) <= tol
        # float64 reference of the backward, with the ReLU' masks and argmaxes
        # of the GPU forward's own output (bf16 operands move values across 0
        # and near-ties): dpre = (y > 0) (gy + scatter_argmax(gp))
        yc = y.cpu()
        _, idx = F.max_pool2d(yc, 2, return_indices=True)
        scat = torch.zeros(F_, cout, hw * hw, dtype=torch.float64)
        scat.scatter_(2, idx.view(F_, cout, -1), gp.double().cpu().view(F_, cout, -1))
        dpre = (yc > 0) * (gy.double().cpu() + scat.view(F_, cout, hw, hw))
        rdx = torch.nn.grad.conv2d_input(xd.shape, wd, dpre, padding=1) * (x.cpu() > 0)
        rdw = torch.nn.grad.conv2d_weight(xd, wd.shape, dpre, padding=1)
        rdb = dpre.sum((0, 2, 3))
        dx = torch.full((F_, cin, hw, hw), float("nan"), device=DEV)
        slab = torch.empty(nmax * (cout * cin * 9 + cout), device=DEV)
        nb = ctypes.c_int(0)
        L().paig_conv2d_bwd(p(x), cin * hw * hw, 0, 0, p(gy), cout * hw * hw, p(dx), cin * hw * hw, p(x),
                            cin * hw * hw, p(w), p(slab), nmax, ctypes.byref(nb), F_, cin, cout, hw, hw, 3,
                            mode | 64 | 2, p(xmax) if mode == 128 else None, XMAX_SLOTS if mode == 128 else 0,
                            p(gp), cout * hp * hp, p(code), cfs, None, st())
        g = torch.empty(cout * cin * 9 + cout, device=DEV)
        L().paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st())
        torch.cuda.synchronize()
        n = cout * cin * 9
        assert torch.isfinite(dx).all()
        assert rel_err(dx, rdx) <= tol, ("dx", F_)
        assert rel_err(g[:n].view_as(w), rdw) <= tol, ("dw", F_)
        assert rel_err(g[n:], rdb) <= 1e-5, ("db", F_)
