"""Per-kernel timing of the U-Net conv kernels at a training step's shapes
(HIP events around N back-to-back launches on one stream).

usage: python tools/conv_bench.py [frames=1000] [modes=split,fp32] [reps=20] [layers=c1,c2,...] [passes=fwd,dgrad,wgrad]
Prints one line per (layer shape, pass, mode): microseconds per launch and the
algorithmic HBM bytes/FLOPs rate of that launch.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paig_reproduction_amd._lib import lib  # noqa: E402

XS = int(os.environ.get("PAIG_XMAX_SLOTS", "2048"))
MODES = {"split": 128, "fp32": 0, "bf16": 256}
# (name, Cin, Cout, H, ks, fused-upsample input): ShallowUNet(hidden 8) at 32x32
LAYERS = [("c1", 3, 8, 32, 3, 0), ("c2", 8, 8, 32, 3, 0), ("c3", 8, 16, 16, 3, 0), ("c4", 16, 16, 16, 3, 0),
          ("c5", 16, 32, 8, 3, 0), ("c6", 32, 32, 8, 3, 0), ("c7", 32, 16, 16, 3, 1), ("c8", 32, 16, 16, 3, 0),
          ("c9", 16, 16, 16, 3, 0), ("c10", 16, 16, 32, 3, 1), ("c11", 24, 8, 32, 3, 0), ("c12", 8, 8, 32, 3, 0),
          ("c13", 8, 2, 32, 1, 0)]
# UNet(hidden 16) at 64x64 (mnist), selected as u1 .. u18
LAYERS += [("u%d" % (i + 1),) + l for i, l in enumerate([
    (3, 16, 64, 3, 0), (16, 16, 64, 3, 0), (16, 32, 32, 3, 0), (32, 32, 32, 3, 0), (32, 64, 16, 3, 0),
    (64, 64, 16, 3, 0), (64, 128, 8, 3, 0), (128, 128, 8, 3, 0), (128, 32, 16, 3, 1), (96, 64, 16, 3, 0),
    (64, 64, 16, 3, 0), (64, 32, 32, 3, 1), (64, 32, 32, 3, 0), (32, 32, 32, 3, 0), (32, 32, 64, 3, 1),
    (48, 16, 64, 3, 0), (16, 16, 64, 3, 0), (16, 2, 64, 1, 0)])]


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    modes = (sys.argv[2] if len(sys.argv) > 2 else "split,fp32").split(",")
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    only = set(sys.argv[4].split(",")) if len(sys.argv) > 4 else None
    passes = set(sys.argv[5].split(",")) if len(sys.argv) > 5 else {"fwd", "dgrad", "wgrad"}
    L = lib()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for name, cin, cout, H, ks, up in LAYERS:
        if only and name not in only:
            continue
        Hin = H // 2 if up else H
        x = torch.rand(F, cin, Hin, Hin, device=dev)
        dy = torch.randn(F, cout, H, H, device=dev)
        w = torch.randn(cout, cin, ks, ks, device=dev) * 0.2
        b = torch.randn(cout, device=dev)
        y = torch.empty(F, cout, H, H, device=dev)
        dx = torch.empty(F, cin, H, H, device=dev)
        aux = torch.rand(F, cin, H, H, device=dev)
        NMAX = int(os.environ.get("PAIG_WG_NMAX", "768"))   # wgrad slab rows (blocks) allowed
        slab = torch.empty(NMAX * (cout * cin * ks * ks + cout), device=dev)
        gsum = torch.empty(cout * cin * ks * ks + cout, device=dev)
        xmax = torch.zeros(XS, device=dev)   # the forward's per-block max |x| slots (ex entry points)
        ex = hasattr(L, "paig_conv2d_fwd_ex")
        nb = ctypes.c_int(0)
        fl = 2 * F * cin * cout * ks * ks * H * H
        for mode in modes:
            m = MODES[mode]
            runs = {
                "fwd": (lambda: L.paig_conv2d_fwd_ex(x.data_ptr(), cin * Hin * Hin, 0, 0, y.data_ptr(), cout * H * H,
                                                     None, 0, w.data_ptr(), b.data_ptr(), F, cin, cout, H, H, ks,
                                                     1 | (32 if up else 0) | m, xmax.data_ptr(), XS, st)) if ex else
                       (lambda: L.paig_conv2d_fwd(x.data_ptr(), cin * Hin * Hin, 0, 0, y.data_ptr(), cout * H * H,
                                                  None, 0, w.data_ptr(), b.data_ptr(), F, cin, cout, H, H, ks,
                                                  1 | (32 if up else 0) | m, st)),
                "wgrad": (lambda: L.paig_conv2d_wgrad_ex(x.data_ptr(), cin * Hin * Hin, 0, 0, dy.data_ptr(),
                                                         cout * H * H, slab.data_ptr(), NMAX, ctypes.byref(nb), F, cin,
                                                         cout, H, H, ks, (32 if up else 0) | m, xmax.data_ptr(), XS,
                                                         st)) if ex else
                         (lambda: L.paig_conv2d_wgrad(x.data_ptr(), cin * Hin * Hin, 0, 0, dy.data_ptr(), cout * H * H,
                                                      slab.data_ptr(), NMAX, ctypes.byref(nb), F, cin, cout, H, H, ks,
                                                      (32 if up else 0) | m, st)),
            }
            # the wgrad with the reduction of its slab rows (the engine batches
            # these into one launch per step; timed here per layer)
            runs["wgred"] = lambda: (runs["wgrad"]() or L.paig_slab_reduce(slab.data_ptr(), nb.value, gsum.numel(),
                                                                            gsum.numel(), gsum.data_ptr(), 0, st))
            if name != "c1":
                runs["dgrad"] = lambda: L.paig_conv2d_fwd(dy.data_ptr(), cout * H * H, 0, 0, dx.data_ptr(),
                                                          cin * H * H, aux.data_ptr(), cin * H * H, w.data_ptr(), None,
                                                          F, cout, cin, H, H, ks, 8 | 2 | m, st)
            for pas, fn in runs.items():
                if pas not in passes:
                    continue
                rc = fn()
                assert rc == 0, (name, pas, mode, L.paig_last_error())
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / reps
                xin = F * cin * Hin * Hin * 4
                byts = {"fwd": xin + F * cout * H * H * 4,
                        "dgrad": F * cout * H * H * 4 + 2 * F * cin * H * H * 4,
                        "wgrad": xin + F * cout * H * H * 4, "wgred": xin + F * cout * H * H * 4}[pas]
                print(f"{name:4s} {pas:5s} {mode:5s} {us:8.1f} us  {byts / us / 1e3:7.0f} GB/s  "
                      f"{fl / us / 1e6:6.1f} TF", flush=True)


if __name__ == "__main__":
    main()
