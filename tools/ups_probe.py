"""Read back the upsampled X image a fused-upsample weight-gradient launch
(paig_conv2d_wgrad_ex, flags 32) stages, through the launch itself: with dY a
one-hot at output channel 0, pixel p of frame f, dW[0][ci][tap] = X_up[ci][p +
tap] (the staged value, scaled back), so one launch per probed pixel reads
every input channel's staged value at the 9 neighbours of p.  Prints the
(channel, position) pairs whose staged value differs from float64
F.interpolate, per channel quad position (ci % 4), for an A/B library
(PAIG_AB_LIB) against the in-tree one.

usage: python tools/ups_probe.py [cin=128] [cout=32] [H=16] [frames=64] [pixels=24]
"""
import ctypes
import os
import sys

import torch
import torch.nn.functional as Fn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paig_reproduction_amd._lib import lib  # noqa: E402

XS = 2048


def main():
    a = [int(v) for v in sys.argv[1:]]
    cin, cout, H, F, npix = (a + [128, 32, 16, 64, 24][len(a):])[:5]
    L = lib()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    torch.manual_seed(1)
    hs = H // 2
    xs = torch.rand(F, cin, hs, hs, device=dev) + 0.5
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.1
    b = torch.zeros(cout, device=dev)
    xmax = torch.zeros(XS, device=dev)
    y = torch.empty(F, cout, H, H, device=dev)
    L.paig_conv2d_fwd_ex(p(xs), cin * hs * hs, 0, 0, p(y), cout * H * H, None, 0, p(w), p(b), F, cin, cout, H, H, 3,
                         32 | 128, p(xmax), XS, st)
    xu = Fn.interpolate(xs.double(), size=(H, H), mode="bilinear", align_corners=False)
    xpad = Fn.pad(xu, (1, 1, 1, 1))
    nmax = 1024
    slab = torch.empty(nmax * (cout * cin * 9 + cout), device=dev)
    g = torch.empty(cout * cin * 9 + cout, device=dev)
    bad = {}
    gen = torch.Generator().manual_seed(3)
    worst = 0.0
    for k in range(npix):
        f = int(torch.randint(F, (1,), generator=gen))
        py, px = int(torch.randint(H, (1,), generator=gen)), int(torch.randint(H, (1,), generator=gen))
        dy = torch.zeros(F, cout, H, H, device=dev)
        dy[f, 0, py, px] = 1.0
        nb = ctypes.c_int(0)
        L.paig_conv2d_wgrad_ex(p(xs), cin * hs * hs, 0, 0, p(dy), cout * H * H, p(slab), nmax, ctypes.byref(nb), F,
                               cin, cout, H, H, 3, 32 | 128, p(xmax), XS, st)
        L.paig_slab_reduce(p(slab), nb.value, g.numel(), g.numel(), p(g), 0, st)
        torch.cuda.synchronize()
        got = g[:cout * cin * 9].view(cout, cin, 3, 3)[0].double().cpu()           # [ci][ty][tx]
        ref = xpad[f, :, py:py + 3, px:px + 3].cpu()                                 # X_up at p + tap
        err = (got - ref).abs()
        worst = max(worst, err.max().item())
        for ci, ty, tx in (err > 1e-5).nonzero().tolist():
            bad.setdefault(ci % 4, []).append((ci, f, py + ty - 1, px + tx - 1, float(got[ci, ty, tx]),
                                               float(ref[ci, ty, tx])))
    print(f"({cin},{cout},{H}) F={F}: {npix} probed pixels, worst staged-value error {worst:.3e}")
    for q in range(4):
        v = bad.get(q, [])
        print(f"  channel % 4 == {q}: {len(v)} wrong staged values", v[:6])


if __name__ == "__main__":
    main()
