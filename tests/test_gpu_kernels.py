"""Per-kernel GPU numerics: each HIP kernel vs a plain PyTorch fp32 CPU
reference of the same op (the aten op the reference calls), at small sizes
including ragged ones.  Bar: 1e-5 normwise for single ops (fp32, different
summation order), unless stated."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_err

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def L():
    from paig_reproduction_amd._lib import lib
    return lib()


def st():
    return torch.cuda.current_stream().cuda_stream


def p(t):
    return None if t is None else t.data_ptr()


CONV_CASES = [(3, 8, 32, 3, 5), (8, 8, 32, 3, 3), (8, 16, 16, 3, 7), (16, 16, 16, 3, 4), (16, 32, 8, 3, 9),
              (32, 32, 8, 3, 3), (32, 16, 16, 3, 2), (24, 8, 32, 3, 2), (8, 2, 32, 1, 3), (16, 16, 32, 3, 2),
              (8, 16, 18, 3, 3), (16, 32, 9, 3, 5), (3, 8, 36, 3, 2),
              # UNet (mnist, 64x64, hidden 16): wide layers, VALU path, combos split over blocks
              (16, 16, 64, 3, 2), (48, 16, 64, 3, 2), (96, 64, 16, 3, 2), (64, 128, 8, 3, 3), (128, 128, 8, 3, 2),
              (16, 2, 64, 1, 2)]


@pytest.mark.parametrize("cin,cout,hw,ks,F_", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(cin, cout, hw, ks, F_):
    torch.manual_seed(cin * 100 + cout)
    x = torch.randn(F_, cin, hw, hw)
    w = torch.randn(cout, cin, ks, ks) * 0.2
    b = torch.randn(cout)
    dy = torch.randn(F_, cout, hw, hw)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, br, padding="same")
    y.backward(dy)
    ref_relu = torch.relu(y.detach())
    xg, wg, bg, dyg = x.to(DEV), w.to(DEV), b.to(DEV), dy.to(DEV)
    out = torch.empty(F_, cout, hw, hw, device=DEV)
    L().paig_conv2d_fwd(p(xg), cin * hw * hw, 0, 0, p(out), cout * hw * hw, None, 0, p(wg), p(bg), F_, cin, cout, hw,
                        hw, ks, 1, st())
    torch.cuda.synchronize()
    assert rel_err(out, ref_relu) <= 1e-5
    # dgrad with ReLU' mask of an activation aux
    aux = torch.relu(torch.randn(F_, cin, hw, hw))
    dx = torch.empty(F_, cin, hw, hw, device=DEV)
    auxg = aux.to(DEV)
    L().paig_conv2d_fwd(p(dyg), cout * hw * hw, 0, 0, p(dx), cin * hw * hw, p(auxg), cin * hw * hw, p(wg), None, F_,
                        cout, cin, hw, hw, ks, 8 | 2, st())
    torch.cuda.synchronize()
    assert rel_err(dx, xr.grad * (aux > 0)) <= 1e-5
    # wgrad
    nmax = 64
    slab = torch.empty(nmax * (cout * cin * ks * ks + cout), device=DEV)
    nb = ctypes.c_int(0)
    L().paig_conv2d_wgrad(p(xg), cin * hw * hw, 0, 0, p(dyg), cout * hw * hw, p(slab), nmax, ctypes.byref(nb), F_, cin,
                          cout, hw, hw, ks, 0, st())
    g = torch.empty(cout * cin * ks * ks + cout, device=DEV)
    L().paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st())
    torch.cuda.synchronize()
    n = cout * cin * ks * ks
    assert rel_err(g[:n].view_as(w), wr.grad) <= 1e-5
    assert rel_err(g[n:], br.grad) <= 1e-5


SPLIT_CASES = [(3, 8, 32, 3, 5), (8, 8, 32, 3, 3), (8, 16, 16, 3, 7), (16, 16, 16, 3, 4), (16, 32, 8, 3, 9),
               (32, 32, 8, 3, 3), (32, 16, 16, 3, 2), (24, 8, 32, 3, 2), (8, 2, 32, 1, 3), (16, 16, 32, 3, 2),
               (16, 8, 16, 3, 3), (8, 24, 32, 3, 2), (2, 8, 32, 1, 3), (32, 16, 8, 3, 3), (16, 32, 16, 3, 2),
               # 3bp (36 x 36 frames): ragged widths 36 / 18 / 9, multi-frame tiles, odd frame counts
               (3, 8, 36, 3, 3), (8, 8, 36, 3, 2), (8, 16, 18, 3, 5), (16, 16, 18, 3, 3), (16, 32, 9, 3, 7),
               (32, 32, 9, 3, 4), (32, 16, 18, 3, 3), (16, 16, 36, 3, 2), (24, 8, 36, 3, 2), (8, 3, 36, 1, 3),
               (16, 8, 18, 3, 3), (32, 16, 9, 3, 5), (16, 32, 18, 3, 2), (8, 24, 36, 3, 2), (3, 8, 36, 1, 2),
               # mnist UNet (64 x 64, 3..128 channels): COUT-sliced forward blocks, smaller pixel tiles,
               # channel-sliced wgrad blocks
               (3, 16, 64, 3, 2), (16, 16, 64, 3, 2), (16, 32, 32, 3, 3), (32, 32, 32, 3, 2), (32, 64, 16, 3, 3),
               (64, 64, 16, 3, 3), (64, 128, 8, 3, 5), (128, 128, 8, 3, 3), (96, 64, 16, 3, 2), (64, 32, 32, 3, 2),
               (48, 16, 64, 3, 2), (16, 2, 64, 1, 2)]
# normwise bars: f16 hi/lo forward ~2^-22 per product (fp32-level); bf16 hi/lo
# dgrad/wgrad ~2^-17; bf16 (hi only) ~2^-9
SPLIT_TOL = {128: (1e-5, 3e-5), 256: (8e-3, 8e-3)}


@pytest.mark.parametrize("mode", [128, 256])
@pytest.mark.parametrize("cin,cout,hw,ks,F_", SPLIT_CASES)
def test_conv_split(cin, cout, hw, ks, F_, mode):
    """Split-precision 16-bit MFMA convs (conv_split.hip) vs torch fp32."""
    tf, tb = SPLIT_TOL[mode]
    torch.manual_seed(cin * 100 + cout + mode)
    x = torch.randn(F_, cin, hw, hw)
    w = torch.randn(cout, cin, ks, ks) * 0.2
    b = torch.randn(cout)
    dy = torch.randn(F_, cout, hw, hw)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, br, padding="same")
    y.backward(dy)
    xg, wg, bg, dyg = x.to(DEV), w.to(DEV), b.to(DEV), dy.to(DEV)
    assert L().paig_conv2d_mfma_supported(0, cin, cout, hw, hw, ks, mode) == 1
    out = torch.empty(F_, cout, hw, hw, device=DEV)
    L().paig_conv2d_fwd(p(xg), cin * hw * hw, 0, 0, p(out), cout * hw * hw, None, 0, p(wg), p(bg), F_, cin, cout, hw,
                        hw, ks, 1 | mode, st())
    torch.cuda.synchronize()
    assert rel_err(out, torch.relu(y.detach())) <= tf
    if L().paig_conv2d_mfma_supported(0, cout, cin, hw, hw, ks, mode | 8):
        aux = torch.relu(torch.randn(F_, cin, hw, hw))
        auxg = aux.to(DEV)
        dx = torch.full((F_, cin, hw, hw), 0.5, device=DEV)
        L().paig_conv2d_fwd(p(dyg), cout * hw * hw, 0, 0, p(dx), cin * hw * hw, p(auxg), cin * hw * hw, p(wg), None,
                            F_, cout, cin, hw, hw, ks, 8 | 4 | 2 | mode, st())
        torch.cuda.synchronize()
        assert rel_err(dx, (xr.grad + 0.5) * (aux > 0)) <= tb
    if L().paig_conv2d_mfma_supported(1, cin, cout, hw, hw, ks, mode):
        nmax = 64
        slab = torch.empty(nmax * (cout * cin * ks * ks + cout), device=DEV)
        nb = ctypes.c_int(0)
        L().paig_conv2d_wgrad(p(xg), cin * hw * hw, 0, 0, p(dyg), cout * hw * hw, p(slab), nmax, ctypes.byref(nb), F_,
                              cin, cout, hw, hw, ks, mode, st())
        g = torch.empty(cout * cin * ks * ks + cout, device=DEV)
        L().paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st())
        torch.cuda.synchronize()
        n = cout * cin * ks * ks
        assert rel_err(g[:n].view_as(w), wr.grad) <= tb
        assert rel_err(g[n:], br.grad) <= 1e-5


@pytest.mark.parametrize("mode", [128, 256])
@pytest.mark.parametrize("cin,cout,hw", [(32, 16, 16), (16, 16, 32), (32, 16, 18), (16, 16, 36), (128, 32, 16),
                                         (64, 32, 32), (32, 32, 64)])
def test_conv_split_fused_upsample(cin, cout, hw, mode):
    """c7/c10: the conv input is the 2x bilinear upsample, formed while staging."""
    tf, tb = SPLIT_TOL[mode]
    torch.manual_seed(cin + cout + hw)
    F_ = 3
    xs = torch.randn(F_, cin, hw // 2, hw // 2)
    xu = F.interpolate(xs, size=(hw, hw), mode="bilinear", align_corners=False, antialias=True)
    w = torch.randn(cout, cin, 3, 3) * 0.2
    b = torch.randn(cout)
    dy = torch.randn(F_, cout, hw, hw)
    xr = xu.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, b, padding="same")
    y.backward(dy)
    xg, wg, bg, dyg = xs.to(DEV), w.to(DEV), b.to(DEV), dy.to(DEV)
    out = torch.empty(F_, cout, hw, hw, device=DEV)
    L().paig_conv2d_fwd(p(xg), cin * hw * hw // 4, 0, 0, p(out), cout * hw * hw, None, 0, p(wg), p(bg), F_, cin, cout,
                        hw, hw, 3, 32 | mode, st())
    nmax = 64
    slab = torch.empty(nmax * (cout * cin * 9 + cout), device=DEV)
    nb = ctypes.c_int(0)
    L().paig_conv2d_wgrad(p(xg), cin * hw * hw // 4, 0, 0, p(dyg), cout * hw * hw, p(slab), nmax, ctypes.byref(nb),
                          F_, cin, cout, hw, hw, 3, 32 | mode, st())
    g = torch.empty(cout * cin * 9 + cout, device=DEV)
    L().paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st())
    torch.cuda.synchronize()
    assert rel_err(out, y.detach()) <= tf
    assert rel_err(g[:cout * cin * 9].view_as(w), wr.grad) <= tb
    # the conv's dgrad (into the upsampled tensor's gradient; the upsample
    # backward is a separate kernel)
    if L().paig_conv2d_mfma_supported(0, cout, cin, hw, hw, 3, mode | 8):
        dx = torch.empty(F_, cin, hw, hw, device=DEV)
        L().paig_conv2d_fwd(p(dyg), cout * hw * hw, 0, 0, p(dx), cin * hw * hw, None, 0, p(wg), None, F_, cout, cin,
                            hw, hw, 3, 8 | mode, st())
        torch.cuda.synchronize()
        assert rel_err(dx, xr.grad) <= tb


def test_conv_split_fused_upsample_many_tiles():
    """c15's fused-upsample forward (window in the lo image's LDS, two blocks
    per CU) with every persistent block walking many tiles: vs float64."""
    tf, _ = SPLIT_TOL[128]
    cin, cout, hw, F_ = 32, 32, 64, 200
    torch.manual_seed(5)
    xs = torch.relu(torch.randn(F_, cin, hw // 2, hw // 2))
    w = torch.randn(cout, cin, 3, 3) * 0.2
    b = torch.randn(cout)
    xu = F.interpolate(xs.double(), size=(hw, hw), mode="bilinear", align_corners=False)
    y = F.conv2d(xu, w.double(), b.double(), padding=1)
    xg, wg, bg = xs.to(DEV), w.to(DEV), b.to(DEV)
    out = torch.empty(F_, cout, hw, hw, device=DEV)
    L().paig_conv2d_fwd(p(xg), cin * hw * hw // 4, 0, 0, p(out), cout * hw * hw, None, 0, p(wg), p(bg), F_, cin, cout,
                        hw, hw, 3, 32 | 128, st())
    torch.cuda.synchronize()
    assert rel_err(out.double().cpu(), y) <= tf


def test_conv_grouped_input_view():
    """The first conv reads frames (b, t < Te) of a [B, T, C, H, W] input in place."""
    B, T, Te, H = 3, 7, 4, 32
    x = torch.rand(B, T, 3, H, H)
    w = torch.randn(8, 3, 3, 3) * 0.3
    b = torch.randn(8)
    ref = torch.relu(F.conv2d(x[:, :Te].reshape(B * Te, 3, H, H), w, b, padding="same"))
    xg, wg, bg = x.to(DEV), w.to(DEV), b.to(DEV)   # keep every operand alive until the kernel ran
    out = torch.empty(B * Te, 8, H, H, device=DEV)
    L().paig_conv2d_fwd(p(xg), T * 3 * H * H, Te, 3 * H * H, p(out), 8 * H * H, None, 0, p(wg), p(bg),
                        B * Te, 3, 8, H, H, 3, 1, st())
    torch.cuda.synchronize()
    assert rel_err(out, ref) <= 1e-5


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(37, 50, 19), (130, 200, 3072), (200, 3072, 130), (6, 2, 200), (1, 513, 200)])
def test_gemm(ta, tb, M, N, K):
    torch.manual_seed(M + N + K)
    A = (torch.randn(K, M) if ta else torch.randn(M, K)) / K ** 0.5   # O(1) pre-activations
    Bm = torch.randn(N, K) if tb else torch.randn(K, N)
    bias = torch.randn(N)
    ref = (A.t() if ta else A) @ (Bm.t() if tb else Bm) + bias
    ref = torch.tanh(ref)
    Ag, Bg, biasg = A.to(DEV), Bm.to(DEV), bias.to(DEV)
    C = torch.empty(M, N, device=DEV)
    ws = torch.empty(max(1, L().paig_gemm_workspace(M, N, K)), device=DEV)
    rs = torch.empty(M, device=DEV)
    L().paig_gemm(ta, tb, M, N, K, 1.0, p(Ag), A.shape[1], p(Bg), Bm.shape[1], 0.0, p(C), N, p(biasg), 2, 0,
                  None, 0, p(rs), p(ws), ws.numel(), st())
    torch.cuda.synchronize()
    assert rel_err(C, ref) <= 2e-5
    assert rel_err(rs, (A.t() if ta else A).sum(1)) <= 2e-5


# split-precision GEMM (paig_gemm_ex): math 1 f16 hi/lo, 2 bf16 hi/lo, 3 bf16,
# 4 f16 hi/lo with op(A) scaled by running powers of two (op(B) fixed 2^8),
# 5 both fixed, 6 both running
GEMM_EX_TOL = {1: 2e-5, 2: 5e-5, 3: 3e-2, 4: 2e-5, 5: 2e-5, 6: 2e-5}


@pytest.mark.parametrize("math", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(37, 50, 19), (130, 200, 3072), (200, 3072, 130), (6, 2, 200), (1, 513, 200),
                                   (2000, 200, 3072), (200, 3072, 2000),    # float4 split-K epilogue
                                   (2000, 3072, 200), (600, 136, 1000)])    # + the 64x256 / 256x64 wide tiles
def test_gemm_ex(ta, tb, M, N, K, math):
    torch.manual_seed(M + N + K + math)
    A = (torch.randn(K, M) if ta else torch.randn(M, K)) / K ** 0.5
    Bm = torch.randn(N, K) if tb else torch.randn(K, N)
    bias = torch.randn(N)
    ref = torch.tanh((A.t() if ta else A) @ (Bm.t() if tb else Bm) + bias)
    Ag, Bg, biasg = A.to(DEV), Bm.to(DEV), bias.to(DEV)
    C = torch.empty(M, N, device=DEV)
    ws = torch.empty(max(1, L().paig_gemm_workspace(M, N, K)), device=DEV)
    rs = torch.full((M,), 7.0, device=DEV)
    rc = L().paig_gemm_ex(ta, tb, M, N, K, 1.0, p(Ag), A.shape[1], p(Bg), Bm.shape[1], 0.0, p(C), N, p(biasg), 2, 0,
                          None, 0, p(rs) if ta else None, p(ws), ws.numel(), math, st())
    torch.cuda.synchronize()
    assert rc == 0
    assert rel_err(C, ref) <= GEMM_EX_TOL[math]
    if ta:   # fused row sums of op(A) in exact fp32
        assert rel_err(rs, A.t().sum(1)) <= 2e-5


# The encoder projection's three products as the engine issues them (math 6):
# forward (bias + ReLU, split-K), wgrad (plain sums + fused bias gradient),
# dgrad (no split) -- the LDS-free fragment-image kernels of dense.hip.
# Operand rows spread over 10^-2..10^2 (the per-row exponents / running
# exponents): normwise and per-row bars vs float64.
@pytest.mark.parametrize("form", ["fwd", "fwd_tb0", "wgrad", "dgrad", "dgrad_tb1"])
def test_gemm_dense_forms(form):
    g = torch.Generator().manual_seed(len(form))
    ta, tb, M, N, K, act = {"fwd": (0, 1, 2000, 200, 3072, 1), "fwd_tb0": (0, 0, 1000, 200, 3072, 1),
                            "wgrad": (1, 0, 200, 3072, 2000, 0), "dgrad": (0, 0, 2000, 3072, 200, 0),
                            "dgrad_tb1": (0, 1, 1500, 3072, 200, 0)}[form]

    def spread(*shape):
        return torch.randn(*shape, generator=g) * 10.0 ** (4 * torch.rand(shape[0], 1, generator=g) - 2)
    A = spread(K, M) if ta else spread(M, K)
    Bm = spread(N, K) if tb else spread(K, N)
    bias = torch.randn(N, generator=g) if act else None
    opA, opB = (A.t() if ta else A).double(), (Bm.t() if tb else Bm).double()
    ref = opA @ opB + (bias.double() if act else 0.0)
    if act:
        ref = torch.relu(ref)
    Ag, Bg = A.to(DEV), Bm.to(DEV)
    bg = bias.to(DEV) if act else None
    ws = torch.empty(max(1, L().paig_gemm_workspace(M, N, K)), device=DEV)
    rs = torch.full((M,), float("nan"), device=DEV)
    outs = []
    for _ in range(2):
        C = torch.full((M, N), float("nan"), device=DEV)
        rc = L().paig_gemm_ex(ta, tb, M, N, K, 1.0, p(Ag), A.shape[1], p(Bg), Bm.shape[1], 0.0, p(C), N,
                              p(bg) if act else None, act, 0, None, 0, p(rs) if ta else None, p(ws), ws.numel(), 6,
                              st())
        torch.cuda.synchronize()
        assert rc == 0, L().paig_last_error()
        outs.append(C.cpu())
    assert torch.equal(outs[0], outs[1]), "not deterministic"
    C = outs[0].double()
    assert rel_err(C, ref) <= 2e-5
    # per output row, against that row's own magnitude (rows whose reference is all ReLU-zero skipped)
    rn = ref.abs().amax(1)
    ok = rn > 0
    assert float(((C - ref).abs().amax(1)[ok] / rn[ok]).max()) <= 1e-4
    if ta:
        assert rel_err(rs.cpu().double(), opA.sum(1)) <= 2e-5


def test_pool_upsample():
    x = torch.relu(torch.randn(5, 6, 16, 16))
    xg = x.to(DEV)
    y = torch.empty(5, 6, 8, 8, device=DEV)
    L().paig_maxpool2_fwd(p(xg), 6 * 256, p(y), 6 * 64, 5, 6, 16, 16, st())
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 2)
    dyy = torch.randn_like(yr)
    yr.backward(dyy)
    base = torch.randn(5, 6, 16, 16)
    dx = base.to(DEV).clone()
    dyg = dyy.to(DEV)
    L().paig_maxpool2_bwd_relu(p(xg), 6 * 256, p(dyg), 6 * 64, p(dx), 6 * 256, 5, 6, 16, 16, st())
    torch.cuda.synchronize()
    assert rel_err(y, yr.detach()) == 0.0
    assert rel_err(dx, (base + xr.grad) * (x > 0)) <= 1e-6
    # upsample 8 -> 16
    s = torch.relu(torch.randn(4, 5, 8, 8))
    sr = s.clone().requires_grad_(True)
    u = F.interpolate(sr, size=(16, 16), mode="bilinear", align_corners=False, antialias=True)
    du = torch.randn_like(u)
    u.backward(du)
    ug = torch.empty(4, 5, 16, 16, device=DEV)
    sg = s.to(DEV)
    L().paig_upsample2_fwd(p(sg), 5 * 64, p(ug), 5 * 256, 4, 5, 8, 8, 16, 16, st())
    ds = torch.empty(4, 5, 8, 8, device=DEV)
    dug = du.to(DEV)
    L().paig_upsample2_bwd(p(dug), 5 * 256, p(sg), 5 * 64, p(ds), 5 * 64, 4, 5, 8, 8, 16, 16, 1, st())
    torch.cuda.synchronize()
    assert rel_err(ug, u.detach()) <= 1e-6
    assert rel_err(ds, sr.grad * (s > 0)) <= 1e-6


@pytest.mark.parametrize("lens,aligned", [([5120, 4096, 36, 0], True), ([64, 100, 7], False), ([3, 8], True)])
@pytest.mark.parametrize("accumulate", [0, 1])
def test_slab_reduce_multi(lens, aligned, accumulate):
    """Batched deterministic slab reductions (vector kernel when every task is
    float4-shaped and aligned, scalar kernel otherwise) vs a float64 sum."""
    g = torch.Generator().manual_seed(7)
    nblks = [1, 300, 129, 2][:len(lens)]
    srcs, dsts, init = [], [], []
    for ln, nb in zip(lens, nblks):
        off = 0 if aligned else 1
        s = torch.randn(nb * ln + off, generator=g)
        d = torch.randn(ln + off, generator=g)
        srcs.append((s.to(DEV), off, s[off:].view(nb, ln) if ln else s[off:].view(nb, 0)))
        dsts.append((d.to(DEV), off))
        init.append(d[off:].clone())
    n = len(lens)
    L().paig_slab_reduce_multi(n, (ctypes.c_void_p * n)(*[p(s) + o * 4 for s, o, _ in srcs]),
                               (ctypes.c_int * n)(*nblks), (ctypes.c_int * n)(*lens),
                               (ctypes.c_void_p * n)(*[p(d) + o * 4 for d, o in dsts]), accumulate, st())
    torch.cuda.synchronize()
    for (d, o), (_, _, host), d0 in zip(dsts, srcs, init):
        want = host.double().sum(0) + (d0.double() if accumulate else 0)
        got = d.cpu()[o:].double()
        assert got.shape == want.shape
        if want.numel():
            assert float((got - want).abs().max()) <= 1e-4 * max(1.0, float(want.abs().max()))


# ---- range: activations, gradients and weights (power-of-two scales from
# their own maxima: per tile, per block, per output channel) work at any
# magnitude, including beyond f16's 65504; the device range flag is raised
# only by a wgrad called without the forward's xmax slots (fixed 2^8 for X)
# and GEMM math 1 (unscaled) beyond 65504
XMAX_SLOTS = 2048


def _range_status():
    return L().paig_f16_range_status(1)


def _split_conv_all(x, w, b, dy, ks, xmax_mode):
    """forward (recording xmax), dgrad, wgrad (X scale from: "fwd" the
    forward's slots, "host" one host-computed slot, "none" the fixed 2^8)"""
    F_, cin, hw = x.shape[0], x.shape[1], x.shape[2]
    cout = w.shape[0]
    xg, wg, bg, dyg = x.to(DEV), w.to(DEV), b.to(DEV), dy.to(DEV)
    out = torch.empty(F_, cout, hw, hw, device=DEV)
    xmax = torch.full((XMAX_SLOTS,), float("nan"), device=DEV)
    L().paig_conv2d_fwd_ex(p(xg), cin * hw * hw, 0, 0, p(out), cout * hw * hw, None, 0, p(wg), p(bg), F_, cin, cout,
                           hw, hw, ks, 128, p(xmax), XMAX_SLOTS, st())
    dx = torch.empty(F_, cin, hw, hw, device=DEV)
    L().paig_conv2d_fwd(p(dyg), cout * hw * hw, 0, 0, p(dx), cin * hw * hw, None, 0, p(wg), None, F_, cout, cin, hw,
                        hw, ks, 8 | 128, st())
    nmax = 64
    slab = torch.empty(nmax * (cout * cin * ks * ks + cout), device=DEV)
    nb = ctypes.c_int(0)
    if xmax_mode == "host":
        xs = torch.zeros(4, device=DEV)
        xs[0] = x.abs().max()
        xp, xn = p(xs), 4
    else:
        xp, xn = (p(xmax), XMAX_SLOTS) if xmax_mode == "fwd" else (None, 0)
    L().paig_conv2d_wgrad_ex(p(xg), cin * hw * hw, 0, 0, p(dyg), cout * hw * hw, p(slab), nmax, ctypes.byref(nb), F_,
                             cin, cout, hw, hw, ks, 128, xp, xn, st())
    g = torch.empty(cout * cin * ks * ks + cout, device=DEV)
    L().paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st())
    torch.cuda.synchronize()
    return out, dx, g[:cout * cin * ks * ks].view_as(w), xmax


@pytest.mark.parametrize("act_scale,dy_scale", [(40.0, 1.0), (1e-5, 1e-12), (1.0, 1e9), (30.0, 1e-20), (1e5, 1.0),
                                                (3e4, 1e6)])
def test_conv_split_any_range(act_scale, dy_scale):
    """Activations and gradients at any magnitude (per-tile / running / the
    forward-recorded power-of-two scales) keep fp32 accuracy, down to f16's
    subnormals and past its 65504 (reference: float64 conv2d)."""
    cin, cout, hw, ks, F_ = 16, 16, 16, 3, 5
    _range_status()
    torch.manual_seed(5)
    x = torch.randn(F_, cin, hw, hw) * act_scale
    w = torch.randn(cout, cin, ks, ks) * 0.2
    b = torch.randn(cout) * act_scale
    dy = torch.randn(F_, cout, hw, hw) * dy_scale
    xr, wr = x.clone().double().requires_grad_(True), w.clone().double().requires_grad_(True)
    y = F.conv2d(xr, wr, b.double(), padding="same")
    y.backward(dy.double())
    for mode in ("fwd", "host"):
        out, dx, gw, xmax = _split_conv_all(x, w, b, dy, ks, mode)
        assert rel_err(out, y.detach()) <= 1e-5
        assert rel_err(dx, xr.grad) <= 1e-5
        assert rel_err(gw, wr.grad) <= 1e-5, mode
        assert _range_status() == 0
    # the slots: every one written, their max = max |x|
    assert torch.isfinite(xmax).all() and float(xmax.max()) == float(x.abs().max())


def test_conv_split_xmax_fallback_flag():
    """A wgrad without the forward's slots stages X at the fixed 2^8: exact
    below 256, flagged (not wrapped) beyond; the forward itself takes any
    magnitude."""
    cin, cout, hw, ks, F_ = 8, 8, 32, 3, 2
    torch.manual_seed(3)
    x = torch.rand(F_, cin, hw, hw) * 100
    w = torch.randn(cout, cin, 3, 3) * 0.2
    b = torch.zeros(cout)
    dy = torch.randn(F_, cout, hw, hw)
    xr, wr = x.clone().double(), w.clone().double().requires_grad_(True)
    F.conv2d(xr, wr, padding="same").backward(dy.double())
    _range_status()
    out, dx, gw, _ = _split_conv_all(x, w, b, dy, ks, "none")
    assert rel_err(gw, wr.grad) <= 1e-5
    assert _range_status() == 0
    x[1, 2, 3, 4] = 1e4
    out, dx, gw, _ = _split_conv_all(x, w, b, dy, ks, "fwd")
    assert rel_err(out, F.conv2d(x.double(), w.double(), padding="same")) <= 1e-5
    assert _range_status() == 0
    _split_conv_all(x, w, b, dy, ks, "none")
    assert _range_status() == 1


@pytest.mark.parametrize("wscale", [1e3, 3e-4])
def test_conv_split_weight_any_range(wscale):
    """Conv weights get a power-of-two exponent per output channel (in-kernel
    staging and paig_conv_wprep images alike): weights up to 1e3 (and tiny
    ones), channels of very different magnitude, match fp64 conv2d at the
    split bars, forward and dgrad, and raise no range flag."""
    cin, cout, hw, ks, F_ = 16, 16, 16, 3, 3
    _range_status()
    torch.manual_seed(11)
    x = torch.rand(F_, cin, hw, hw)
    w = torch.randn(cout, cin, ks, ks) * wscale
    w[3] *= 1e-4          # a channel far below the others
    w[5, 2, 1, 1] = 3.0 * wscale
    b = torch.randn(cout)
    dy = torch.randn(F_, cout, hw, hw)
    xr, wr = x.clone().double().requires_grad_(True), w.clone().double()
    y = F.conv2d(xr, wr, b.double(), padding="same")
    y.backward(dy.double())
    xg, wg, bg, dyg = x.to(DEV), w.to(DEV), b.to(DEV), dy.to(DEV)
    # in-kernel staging
    out = torch.empty(F_, cout, hw, hw, device=DEV)
    L().paig_conv2d_fwd(p(xg), cin * hw * hw, 0, 0, p(out), cout * hw * hw, None, 0, p(wg), p(bg), F_, cin, cout, hw,
                        hw, ks, 128, st())
    dx = torch.empty(F_, cin, hw, hw, device=DEV)
    L().paig_conv2d_fwd(p(dyg), cout * hw * hw, 0, 0, p(dx), cin * hw * hw, None, 0, p(wg), None, F_, cout, cin, hw,
                        hw, ks, 8 | 128, st())
    torch.cuda.synchronize()
    assert rel_err(out, y.detach()) <= 1e-5
    assert rel_err(dx, xr.grad) <= 1e-5
    # prepped images (the training step's path)
    jobs = [(cin, cout, 0), (cout, cin, 1)]
    sizes = [int(L().paig_conv_wprep_size(a, c, ks)) for a, c, _ in jobs]
    buf = torch.zeros(sum(sizes), dtype=torch.int16, device=DEV)
    outs = [buf.data_ptr(), buf.data_ptr() + 2 * sizes[0]]
    n = len(jobs)
    L().paig_conv_wprep(n, (ctypes.c_void_p * n)(*[p(wg)] * n), (ctypes.c_int * n)(*[j[0] for j in jobs]),
                        (ctypes.c_int * n)(*[j[1] for j in jobs]), (ctypes.c_int * n)(ks, ks),
                        (ctypes.c_int * n)(*[j[2] for j in jobs]), (ctypes.c_void_p * n)(*outs), st())
    out2 = torch.empty_like(out)
    dx2 = torch.empty_like(dx)
    L().paig_conv2d_fwd_pw(p(xg), cin * hw * hw, 0, 0, p(out2), cout * hw * hw, None, 0, p(wg), p(bg), F_, cin, cout,
                           hw, hw, ks, 128, None, 0, None, 0, outs[0], st())
    L().paig_conv2d_fwd_pw(p(dyg), cout * hw * hw, 0, 0, p(dx2), cin * hw * hw, None, 0, p(wg), None, F_, cout, cin,
                           hw, hw, ks, 8 | 128, None, 0, None, 0, outs[1], st())
    torch.cuda.synchronize()
    assert torch.equal(out2, out) and torch.equal(dx2, dx), "prepped images must match in-kernel staging bit for bit"
    assert _range_status() == 0


def test_gemm_math1_range_flag():
    M, N, K = 64, 64, 64
    _range_status()
    A = torch.randn(M, K, device=DEV) * 1e5
    Bm = torch.randn(K, N, device=DEV)
    C = torch.empty(M, N, device=DEV)
    L().paig_gemm_ex(0, 0, M, N, K, 1.0, p(A), K, p(Bm), N, 0.0, p(C), N, None, 0, 0, None, 0, None, None, 0, 1, st())
    assert _range_status() == 1
    # math 4 (op(A) = a gradient, scaled dynamically) at the same magnitude: exact, no flag
    L().paig_gemm_ex(0, 0, M, N, K, 1.0, p(A), K, p(Bm), N, 0.0, p(C), N, None, 0, 0, None, 0, None, None, 0, 4, st())
    torch.cuda.synchronize()
    ref = A.double().cpu() @ Bm.double().cpu()
    assert rel_err(C, ref) <= 2e-5
    assert _range_status() == 0
    # math 6 (both running): op(B) far outside f16 too, and tiny
    for sb in (1e7, 1e-9):
        B2 = Bm * sb
        L().paig_gemm_ex(0, 0, M, N, K, 1.0, p(A), K, p(B2), N, 0.0, p(C), N, None, 0, 0, None, 0, None, None, 0, 6,
                         st())
        torch.cuda.synchronize()
        assert rel_err(C, A.double().cpu() @ B2.double().cpu()) <= 2e-5
        assert _range_status() == 0


@pytest.mark.parametrize("K,hw,F_", [(2, 32, 37), (3, 36, 5)])
def test_head_mask_fused(K, hw, F_):
    """paig_head_mask_fwd/bwd (ShallowUNet c13 1x1 + ReLU, cat(ones), softmax,
    mask x image; blocks.py:84-93,276,307) against the same ops in fp32 torch:
    masks, masked objects, c12's input gradient (c12's ReLU' applied) and
    c13's weight / bias gradients (slab rows summed on the host)."""
    torch.manual_seed(K * 100 + hw)
    HW = hw * hw
    x12 = torch.relu(torch.randn(F_, 8, hw, hw))
    x12[:, :, :3] = 0.0   # dead pixels: ReLU' of c12 must zero them
    img = torch.rand(F_, 3, hw, hw)
    w = torch.randn(K, 8) * 0.5
    b = torch.randn(K) * 0.2
    dobjs = torch.randn(K, F_, 3, hw, hw)
    # reference
    xr = x12.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    lg = torch.relu(F.conv2d(xr, wr.view(K, 8, 1, 1), br))
    masks_ref = torch.softmax(torch.cat([lg, torch.ones(F_, 1, hw, hw)], 1), 1)   # blocks.py:84-90
    objs_ref = torch.stack([masks_ref[:, k:k + 1] * img for k in range(K)], 0)
    (objs_ref * dobjs).sum().backward()
    dx_ref = xr.grad * (x12 > 0)
    # device
    g = {n: t.to(DEV).contiguous() for n, t in dict(x12=x12, img=img, w=w, b=b, dobjs=dobjs).items()}
    masks = torch.empty(F_, K + 1, hw, hw, device=DEV)
    objs = torch.empty(K, F_, 3, hw, hw, device=DEV)
    assert L().paig_head_mask_fwd(p(g["x12"]), p(g["w"]), p(g["b"]), p(g["img"]), 3 * HW, 0, 0, p(masks), p(objs), F_, K,
                                  hw, hw, st()) == 0
    nb = L().paig_head_mask_blocks(F_, hw, hw)
    slab = torch.empty(nb, K * 8 + K, device=DEV)
    dx = torch.empty(F_, 8, hw, hw, device=DEV)
    assert L().paig_head_mask_bwd(p(g["x12"]), p(g["w"]), p(g["b"]), p(g["img"]), 3 * HW, 0, 0, p(masks), p(g["dobjs"]),
                                  p(dx), p(slab), F_, K, hw, hw, st()) == 0
    torch.cuda.synchronize()
    part = slab.sum(0).cpu()
    assert rel_err(masks, masks_ref.detach()) <= 1e-6
    assert rel_err(objs, objs_ref.detach()) <= 1e-6
    assert rel_err(dx, dx_ref) <= 1e-5
    assert rel_err(part[:K * 8].view(K, 8), wr.grad) <= 1e-5
    assert rel_err(part[K * 8:], br.grad) <= 1e-5


@pytest.mark.parametrize("K,hw,F_", [(2, 64, 9), (3, 64, 3), (2, 40, 5)])
def test_head_mask_fused_unet(K, hw, F_):
    """paig_head_mask_fwd_ex/_bwd_ex with the UNet head (c18: 1x1 conv 16 -> K,
    not ReLU'd; cat(ones), softmax, mask x image and the masked objects'
    AvgPool2d(2); blocks.py:84-96,170,236) against the same ops in fp64 torch:
    masks, masked objects, pooled objects, c17's input gradient (c17's ReLU'
    applied) from the pooled objects' gradient, c18's weight / bias gradient."""
    torch.manual_seed(K * 1000 + hw)
    HW = hw * hw
    x17 = torch.relu(torch.randn(F_, 16, hw, hw))
    x17[:, :, :2] = 0.0   # dead pixels: c17's ReLU' must zero them
    img = torch.rand(F_, 3, hw, hw)
    w = torch.randn(K, 16) * 0.4
    b = torch.randn(K) * 0.2
    dpobjs = torch.randn(K, F_, 3, hw // 2, hw // 2)
    xr = x17.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    lg = F.conv2d(xr, wr.view(K, 16, 1, 1), br)   # c18: no ReLU (blocks.py:236)
    masks_ref = torch.softmax(torch.cat([lg, torch.ones(F_, 1, hw, hw, dtype=torch.float64)], 1), 1)
    objs_ref = torch.stack([masks_ref[:, k:k + 1] * img.double() for k in range(K)], 0)
    pobjs_ref = F.avg_pool2d(objs_ref.reshape(K * F_, 3, hw, hw), 2).view(K, F_, 3, hw // 2, hw // 2)
    (pobjs_ref * dpobjs.double()).sum().backward()
    dx_ref = xr.grad * (x17 > 0)
    g = {n: t.to(DEV).contiguous() for n, t in dict(x17=x17, img=img, w=w, b=b, dp=dpobjs).items()}
    masks = torch.empty(F_, K + 1, hw, hw, device=DEV)
    objs = torch.empty(K, F_, 3, hw, hw, device=DEV)
    pobjs = torch.empty(K, F_, 3, hw // 2, hw // 2, device=DEV)
    L().paig_head_mask_fwd_ex(p(g["x17"]), p(g["w"]), p(g["b"]), p(g["img"]), 3 * HW, 0, 0, p(masks), p(objs),
                              p(pobjs), F_, K, 16, hw, hw, 2, st())
    nb = L().paig_head_mask_blocks(F_, hw, hw)
    slab = torch.empty(nb, K * 16 + K, device=DEV)
    dx = torch.full((F_, 16, hw, hw), float("nan"), device=DEV)
    L().paig_head_mask_bwd_ex(p(g["x17"]), p(g["w"]), p(g["b"]), p(g["img"]), 3 * HW, 0, 0, p(masks), p(g["dp"]),
                              p(dx), p(slab), F_, K, 16, hw, hw, 2, st())
    torch.cuda.synchronize()
    part = slab.double().sum(0).cpu()
    assert rel_err(masks, masks_ref.detach()) <= 1e-6
    assert rel_err(objs, objs_ref.detach()) <= 1e-6
    assert rel_err(pobjs, pobjs_ref.detach()) <= 1e-6
    assert torch.isfinite(dx).all()
    assert rel_err(dx, dx_ref) <= 1e-5
    assert rel_err(part[:K * 16].view(K, 16), wr.grad) <= 1e-5
    assert rel_err(part[K * 16:], br.grad) <= 1e-5
    # the (CI, flags) pairs are the two heads only
    with pytest.raises(Exception):
        L().paig_head_mask_fwd_ex(p(g["x17"]), p(g["w"]), p(g["b"]), p(g["img"]), 3 * HW, 0, 0, p(masks), p(objs),
                                  p(pobjs), F_, K, 16, hw, hw, 1, st())


@pytest.mark.parametrize("cin,cout,hw,ks,up", [(8, 8, 32, 3, 0), (32, 32, 8, 3, 0), (24, 8, 32, 3, 0), (8, 24, 32, 3, 0),
                                               (64, 128, 16, 3, 0), (32, 16, 16, 3, 1), (8, 2, 32, 1, 0)])
def test_conv_wprep_bit_identical(cin, cout, hw, ks, up):
    """Split forward / dgrad with weight images from paig_conv_wprep (one
    launch per step) give bit-identical results to the in-kernel staging,
    including a multi-slice COUT (64 -> 128 at 16x16, grid.y > 1)."""
    torch.manual_seed(cin + cout + hw)
    hin = hw // 2 if up else hw
    x = torch.randn(3, cin, hin, hin, device=DEV)
    w = torch.randn(cout, cin, ks, ks, device=DEV) * 0.2
    b = torch.randn(cout, device=DEV)
    dy = torch.randn(3, cout, hw, hw, device=DEV)
    fl = 128 | (32 if up else 0)
    jobs = [(cin, cout, 0)] + ([] if up else [(cout, cin, 1)])
    sizes = [int(L().paig_conv_wprep_size(a, c, ks)) for a, c, _ in jobs]
    bufs = [torch.empty(n, dtype=torch.int16, device=DEV) for n in sizes]
    n = len(jobs)
    L().paig_conv_wprep(n, (ctypes.c_void_p * n)(*[p(w)] * n), (ctypes.c_int * n)(*[j[0] for j in jobs]),
                        (ctypes.c_int * n)(*[j[1] for j in jobs]), (ctypes.c_int * n)(*[ks] * n),
                        (ctypes.c_int * n)(*[j[2] for j in jobs]), (ctypes.c_void_p * n)(*[p(t) for t in bufs]), st())
    outs = []
    for wpp in (None, p(bufs[0])):
        o = torch.empty(3, cout, hw, hw, device=DEV)
        L().paig_conv2d_fwd_pw(p(x), cin * hin * hin, 0, 0, p(o), cout * hw * hw, None, 0, p(w), p(b), 3, cin, cout,
                               hw, hw, ks, 1 | fl, None, 0, None, 0, wpp, st())
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    if not up:
        aux = torch.relu(torch.randn(3, cin, hw, hw, device=DEV))
        dxs = []
        for wpp in (None, p(bufs[1])):
            dx = torch.full((3, cin, hw, hw), 0.5, device=DEV)
            L().paig_conv2d_fwd_pw(p(dy), cout * hw * hw, 0, 0, p(dx), cin * hw * hw, p(aux), cin * hw * hw, p(w), None,
                                   3, cout, cin, hw, hw, ks, 8 | 4 | 2 | 128, None, 0, None, 0, wpp, st())
            dxs.append(dx)
        torch.cuda.synchronize()
        assert torch.equal(dxs[0], dxs[1])


@pytest.mark.parametrize("cin,cout,hw,mode", [(8, 8, 32, 128), (16, 16, 16, 128), (8, 8, 32, 256), (3, 8, 32, 128), (16, 16, 64, 128), (32, 32, 32, 128), (32, 32, 32, 256), (64, 64, 16, 128)])
def test_conv_fused_pool(cin, cout, hw, mode):
    """Split forward with the fused 2x2 max pool (flags & 64): the conv output
    is unchanged and the pooled output is bit-identical to paig_maxpool2_fwd
    on it (aten's window scan order; ReLU zeros and ties included)."""
    torch.manual_seed(cin * 7 + hw)
    F_ = 5
    x = torch.randn(F_, cin, hw, hw, device=DEV)
    w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.2
    b = torch.randn(cout, device=DEV)
    assert L().paig_conv2d_mfma_supported(0, cin, cout, hw, hw, 3, mode | 64) == 1
    h2 = hw // 2
    y0 = torch.empty(F_, cout, hw, hw, device=DEV)
    y1 = torch.empty(F_, cout, hw, hw, device=DEV)
    pool = torch.full((F_, cout, h2, h2), float("nan"), device=DEV)
    ref = torch.empty(F_, cout, h2, h2, device=DEV)
    L().paig_conv2d_fwd_pw(p(x), cin * hw * hw, 0, 0, p(y0), cout * hw * hw, None, 0, p(w), p(b), F_, cin, cout, hw, hw,
                           3, 1 | mode, None, 0, None, 0, None, st())
    L().paig_conv2d_fwd_pw(p(x), cin * hw * hw, 0, 0, p(y1), cout * hw * hw, None, 0, p(w), p(b), F_, cin, cout, hw, hw,
                           3, 1 | mode | 64, None, 0, p(pool), cout * h2 * h2, None, st())
    L().paig_maxpool2_fwd(p(y0), cout * hw * hw, p(ref), cout * h2 * h2, F_, cout, hw, hw, st())
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(pool, ref)
    assert L().paig_conv2d_mfma_supported(0, cin, cout, 36, 36, 3, mode | 64) == 0   # 36-wide rows: no in-lane windows
    # window codes: the fused pool's and the standalone pool's
    # (paig_maxpool2_fwd_codes, 3bp's layers) are the same bytes
    cfs = -(-cout // 8) * 8 * h2 * h2
    c1 = torch.zeros(F_ * cfs, dtype=torch.uint8, device=DEV)
    c2 = torch.ones(F_ * cfs, dtype=torch.uint8, device=DEV)
    pool2 = torch.empty_like(pool)
    L().paig_conv2d_fwd_pwc(p(x), cin * hw * hw, 0, 0, p(y1), cout * hw * hw, None, 0, p(w), p(b), F_, cin, cout, hw,
                            hw, 3, 1 | mode | 64, None, 0, p(pool), cout * h2 * h2, p(c1), cfs, None, st())
    L().paig_maxpool2_fwd_codes(p(y0), cout * hw * hw, p(pool2), cout * h2 * h2, p(c2), cfs, F_, cout, hw, hw, st())
    torch.cuda.synchronize()
    assert torch.equal(pool2, ref)
    if cout % 8 == 0:   # (padding channels of a partial 8-channel group are not written)
        assert torch.equal(c1, c2)


@pytest.mark.parametrize("R", [6, 46, 64, 65, 70])
def test_rollout_spring_adjoint_scan_and_serial(R):
    """paig_rollout_bwd for the spring cell: the Hillis-Steele scan adjoint
    (R <= 64) and the serial one (R > 64) against autograd through a float64
    restatement of the R-step rollout (oracle spring_cell, nn/network/
    cells.py:31-51), with a loss on every step's positions and velocities:
    d pos0, d vel0 and the physics-parameter gradients at 1e-4 normwise."""
    from oracle import physics_oracle as O
    B, D = 37, 4
    g = torch.Generator().manual_seed(R)
    # columns 0 and 1 are the spring's ends (Q3): keep them near the rest
    # length 2 exp(equil) = 6 so the oscillation never passes n = 0, where
    # d = x / (n + 1e-4) has a 1e4 slope and any fp32 trajectory decorrelates
    # from the float64 one
    pos0 = 16 + 2 * (torch.rand(B, D, generator=g) - 0.5)
    sgn = torch.where(torch.rand(B, generator=g) < 0.5, -1.0, 1.0)
    pos0[:, 0] = pos0[:, 1] + sgn * (6 + 2 * (torch.rand(B, generator=g) - 0.5))
    vel0 = (torch.rand(B, D, generator=g) - 0.5)
    dt = torch.tensor(0.3, dtype=torch.float32)
    k = torch.tensor(np.log(4.0), dtype=torch.float64)
    eq = torch.tensor(np.log(3.0), dtype=torch.float64)
    dpos_roll = torch.randn(B, R, D, generator=g)
    dpvs = torch.randn(B, R + 1, 2 * D, generator=g)
    # reference (float64)
    P = {"rollout_cell.dt": dt.double(), "rollout_cell.k": k.clone().requires_grad_(True),
         "rollout_cell.equil": eq.clone().requires_grad_(True)}
    p = pos0.double().requires_grad_(True)
    v = vel0.double().requires_grad_(True)
    loss = (dpvs[:, 0, :D].double() * p).sum() + (dpvs[:, 0, D:].double() * v).sum()
    pc, vc = p, v
    for t in range(R):
        pc, vc = O.spring_cell(P, pc, vc)
        loss = loss + (dpos_roll[:, t].double() * pc).sum() + (dpvs[:, t + 1, :D].double() * pc).sum() \
            + (dpvs[:, t + 1, D:].double() * vc).sum()
    loss.backward()
    # HIP
    dev = DEV
    pvs = torch.empty(B, R + 1, 2 * D, device=dev)
    vk = vel0.view(B, D // 2, 2).permute(1, 0, 2).contiguous().to(dev)
    dtg, kg, eqg = dt.to(dev), k.to(dev), eq.to(dev)
    pg = pos0.to(dev)
    assert L().paig_rollout_fwd(0, p_(pg), D, p_(vk), p_(dtg), p_(kg), p_(eqg), p_(pvs), B, D, R, st()) == 0
    dpos0 = torch.empty(B, D, device=dev)
    dvel0 = torch.empty(D // 2, B, 2, device=dev)
    part = torch.empty(2 * L().paig_rollout_bwd_blocks(B), device=dev, dtype=torch.float64)
    gq = torch.zeros(2, device=dev, dtype=torch.float64)
    dr, dv = dpos_roll.to(dev).contiguous(), dpvs.to(dev).contiguous()
    assert L().paig_rollout_bwd(0, p_(pvs), p_(dr), p_(dv), p_(dtg), p_(kg), p_(eqg), p_(dpos0), p_(dvel0), p_(part),
                                p_(gq), p_(gq) + 8, 0, B, D, R, st()) == 0
    torch.cuda.synchronize()
    assert rel_err(dpos0, p.grad) <= 1e-4, ("dpos0", rel_err(dpos0, p.grad))
    assert rel_err(dvel0.permute(1, 0, 2).reshape(B, D), v.grad) <= 1e-4
    assert rel_err(gq[0:1], P["rollout_cell.k"].grad.view(1)) <= 1e-4
    assert rel_err(gq[1:2], P["rollout_cell.equil"].grad.view(1)) <= 1e-4


def p_(t):
    return t.data_ptr()
