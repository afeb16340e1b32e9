"""Per-launch time of the fused layer backward (csrc/conv_bwd.hip,
paig_conv2d_bwd) at the training step's shapes, HIP events around `reps`
back-to-back launches; with a -DPAIG_BWD_STAMPS library (PAIG_AB_LIB) also the
per-tile phase breakdown in shader cycles (s_memtime sums per wave).

usage: python tools/bwd_bench.py [layers=c10,c11] [frames=1000] [reps=20] [mode=split|bf16]
Layers: the ShallowUNet's c2..c12 at 32 x 32 (spring), u2 / u3 / u17 of the
mnist UNet at 64 x 64 (frames default 2560 there).
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paig_reproduction_amd._lib import lib  # noqa: E402

XS = 2048
# name: (Cin, Cout, H, kind, aux, accumulate); kind: "" | "up" (fused
# upsample input) | "pool" (2x2 max pool of the output folded)
LAYERS = {
    "c2": (8, 8, 32, "pool", 1, 0), "c3": (8, 16, 16, "", 0, 0), "c4": (16, 16, 16, "pool", 1, 0),
    "c5": (16, 32, 8, "", 0, 0), "c6": (32, 32, 8, "", 1, 0), "c7": (32, 16, 16, "up", 1, 0),
    "c8": (32, 16, 16, "", 0, 0), "c9": (16, 16, 16, "", 1, 0), "c10": (16, 16, 32, "up", 1, 0),
    "c11": (24, 8, 32, "", 0, 0), "c12": (8, 8, 32, "", 1, 0),
    "u2": (16, 16, 64, "pool", 1, 0), "u3": (16, 32, 32, "", 0, 0), "u17": (16, 16, 64, "", 1, 0),
}
PHASES = ["setup", "wait+max+bar", "commit-tail", "issue", "wgrad", "dgrad", "epilogue", "slab", "put_d", "ups_win",
          "ups_bar", "ups_x"]


def main():
    names = (sys.argv[1] if len(sys.argv) > 1 else "c2,c4,c7,c9,c10,c11,c12").split(",")
    F0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    mode = {"split": 128, "bf16": 256}[sys.argv[4] if len(sys.argv) > 4 else "split"]
    L = lib()
    stamps = getattr(L.dll, "paig_bwd_stamps_read", None) if hasattr(L.dll, "paig_bwd_stamps_read") else None
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    for nm in names:
        cin, cout, H, kind, aux_on, acc = LAYERS[nm]
        F = F0 or (2560 if H == 64 or nm.startswith("u") else 1000)
        torch.manual_seed(0)
        Hx = H // 2 if kind == "up" else H
        x = torch.relu(torch.randn(F, cin, Hx, Hx, device=dev))
        w = torch.randn(cout, cin, 3, 3, device=dev) * 0.2
        b = torch.randn(cout, device=dev)
        dy = torch.randn(F, cout, H, H, device=dev)
        dx = torch.zeros(F, cin, Hx, Hx, device=dev)
        xmax = torch.zeros(XS, device=dev)
        fl = mode | (32 if kind == "up" else 0)
        y = torch.empty(F, cout, H, H, device=dev)
        hp = H // 2
        pool = code = None
        cfs = 0
        if kind == "pool":
            pool = torch.randn(F, cout, hp, hp, device=dev)
            cfs = -(-cout // 8) * 8 * hp * hp
            code = torch.empty(F * cfs, dtype=torch.uint8, device=dev)
            L.paig_conv2d_fwd_pwc(p(x), cin * H * H, 0, 0, p(y), cout * H * H, None, 0, p(w), p(b), F, cin, cout, H,
                                  H, 3, 1 | 64 | mode, p(xmax) if mode == 128 else None, XS if mode == 128 else 0,
                                  p(pool), cout * hp * hp, p(code), cfs, None, st)
        else:
            L.paig_conv2d_fwd_ex(p(x), cin * Hx * Hx, 0, 0, p(y), cout * H * H, None, 0, p(w), p(b), F, cin, cout, H,
                                 H, 3, fl, p(xmax) if mode == 128 else None, XS if mode == 128 else 0, st)
        n = int(L.paig_conv_wprep_size(cout, cin, 3))
        wp = torch.empty(n, dtype=torch.int16, device=dev)
        L.paig_conv_wprep(1, (ctypes.c_void_p * 1)(p(w)), (ctypes.c_int * 1)(cout), (ctypes.c_int * 1)(cin),
                          (ctypes.c_int * 1)(3), (ctypes.c_int * 1)(1), (ctypes.c_void_p * 1)(p(wp)), st)
        nmax = 1024
        slab = torch.empty(nmax * (cout * cin * 9 + cout), device=dev)
        nb = ctypes.c_int(0)
        flags = fl | (64 if kind == "pool" else 0) | (2 if aux_on else 0) | (4 if acc else 0)

        def run():
            L.paig_conv2d_bwd(p(x), cin * Hx * Hx, 0, 0, p(dy), cout * H * H, p(dx), cin * Hx * Hx,
                              p(x) if aux_on else None, cin * Hx * Hx, p(w), p(slab), nmax, ctypes.byref(nb), F, cin,
                              cout, H, H, 3, flags, p(xmax) if mode == 128 else None, XS if mode == 128 else 0,
                              p(pool), cout * hp * hp, p(code), cfs, p(wp) if mode == 128 else None, st)

        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        byts = 4 * F * (cin * Hx * Hx * (1 + aux_on + 1 + acc) + cout * H * H)
        line = f"{nm:4s} ({cin:3d},{cout:3d},{H:2d},{kind or '-':4s}) F={F:5d} blocks={nb.value:4d} {us:8.1f} us " \
               f"{byts / us / 1e3:7.0f} GB/s"
        if stamps is not None:
            run()
            torch.cuda.synchronize()
            buf = (ctypes.c_ulonglong * (4096 * 4 * 13))()
            stamps(buf, ctypes.sizeof(buf))
            t = torch.tensor(list(buf), dtype=torch.float64).view(4096, 4, 13)[:nb.value]
            tiles = t[:, :, 12].sum().item()
            per = [t[:, :, k].sum().item() / max(tiles, 1) for k in range(12)]
            line += " | cyc/tile " + " ".join(f"{PHASES[k]}={per[k]:.0f}" for k in range(12) if per[k]) + \
                    f" | loop={sum(per[1:7]) + sum(per[8:]):.0f} tiles/blk={tiles / 4 / max(nb.value, 1):.1f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
