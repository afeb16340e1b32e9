"""Bit-identity of the fused-upsample conv kernels between two builds of the
library (e.g. an A/B staging change that must not change a single bit):
forward (paig_conv2d_fwd_ex), weight gradient (paig_conv2d_wgrad_ex) and the
fused layer backward (paig_conv2d_bwd) on the same random operands.

usage: python tools/bitid_check.py <other.so> [frames=64]
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paig_reproduction_amd._lib import LIB_PATH, _Lib  # noqa: E402

XS = 2048
# (Cin, Cout, H): the UNet's c9 / c12 / c15 and the ShallowUNet's c7 / c10
SHAPES = [(128, 32, 16), (64, 32, 32), (32, 32, 64), (32, 16, 16), (16, 16, 32)]


def run(L, cin, cout, H, F, dev):
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(cin * 7 + cout + H)
    hs = H // 2
    xs = torch.relu(torch.randn(F, cin, hs, hs, device=dev))
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.1
    b = torch.randn(cout, device=dev)
    dy = torch.randn(F, cout, H, H, device=dev)
    xmax = torch.zeros(XS, device=dev)
    y = torch.empty(F, cout, H, H, device=dev)
    L.paig_conv2d_fwd_ex(p(xs), cin * hs * hs, 0, 0, p(y), cout * H * H, None, 0, p(w), p(b), F, cin, cout, H, H, 3,
                         32 | 128, p(xmax), XS, st)
    nmax = 1024
    slab = torch.empty(nmax * (cout * cin * 9 + cout), device=dev)
    nb = ctypes.c_int(0)
    L.paig_conv2d_wgrad_ex(p(xs), cin * hs * hs, 0, 0, p(dy), cout * H * H, p(slab), nmax, ctypes.byref(nb), F, cin,
                           cout, H, H, 3, 32 | 128, p(xmax), XS, st)
    gw = torch.empty(cout * cin * 9 + cout, device=dev)
    L.paig_slab_reduce(p(slab), nb.value, gw.numel(), gw.numel(), p(gw), 0, st)
    out = {"fwd": y.clone(), "wgrad": gw.clone()}
    if L.paig_conv2d_bwd_supported(cin, cout, H, H, 3, 128 | 32):
        dx = torch.empty(F, cin, hs, hs, device=dev)
        L.paig_conv2d_bwd(p(xs), cin * hs * hs, 0, 0, p(dy), cout * H * H, p(dx), cin * hs * hs, p(xs), cin * hs * hs,
                          p(w), p(slab), nmax, ctypes.byref(nb), F, cin, cout, H, H, 3, 128 | 32 | 2, p(xmax), XS,
                          None, 0, None, 0, None, st)
        L.paig_slab_reduce(p(slab), nb.value, gw.numel(), gw.numel(), p(gw), 0, st)
        out["bwd_dx"] = dx
        out["bwd_dw"] = gw.clone()
    torch.cuda.synchronize()
    return out


def main():
    other = sys.argv[1]
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    dev = torch.device("cuda:0")
    A, B = _Lib(LIB_PATH), _Lib(other)
    bad = 0
    for cin, cout, H in SHAPES:
        ra, rb = run(A, cin, cout, H, F, dev), run(B, cin, cout, H, F, dev)
        for k in ra:
            same = torch.equal(ra[k], rb[k])
            d = (ra[k] - rb[k]).abs().max().item()
            bad += not same
            print(f"({cin},{cout},{H}) {k:7s} {'bit-identical' if same else f'DIFFERS max |d| {d:.3g}'}", flush=True)
            if not same and k in ("wgrad", "bwd_dw") and d > 1e-3:
                # where: max |d| per tap (ky, kx) and per input channel
                n = cout * cin * 9
                dd = (ra[k] - rb[k])[:n].abs().view(cout, cin, 3, 3)
                print("    per tap:", [[round(dd[:, :, ky, kx].max().item(), 3) for kx in range(3)] for ky in range(3)])
                print("    per cin:", [round(v, 2) for v in dd.amax((0, 2, 3)).tolist()])
                print("    per cout:", [round(v, 2) for v in dd.amax((1, 2, 3)).tolist()])
    print("BITID_OK" if bad == 0 else f"BITID_FAIL {bad}")


if __name__ == "__main__":
    main()
