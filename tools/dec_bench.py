"""Per-launch timing of the decoder kernels (paig_decoder_fwd / _bwd) at the
BASELINE configs' shapes (HIP events around back-to-back launches on one
stream), with the algorithmic bytes of each launch (engine._dec_bwd_bytes).

usage: python tools/dec_bench.py [reps=50] [cases=all|name,name]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paig_reproduction_amd._lib import lib  # noqa: E402

# name: (K, H, B, R or 0 (ungrouped: B frames), live steps)
CASES = {
    "spring_roll": (2, 32, 100, 46, 6), "spring_rec": (2, 32, 1000, 0, 0),
    "spring512_roll": (2, 32, 512, 46, 6), "spring512_rec": (2, 32, 5120, 0, 0),
    "3bp_roll": (3, 36, 512, 16, 12), "3bp_rec": (3, 36, 8192, 0, 0),
    "bounce_roll": (2, 32, 1024, 96, 6), "bounce_rec": (2, 32, 10240, 0, 0),
    "mnist_roll": (2, 64, 256, 9, 7), "mnist_rec": (2, 64, 2560, 0, 0),
}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    want = sys.argv[2].split(",") if len(sys.argv) > 2 and sys.argv[2] != "all" else list(CASES)
    L = lib()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    for name in want:
        K, H, B, R, live = CASES[name]
        h = H // 2
        F = B * R if R else B
        fr = 3 * H * H
        T = (R + 4) if R else 1
        pos = (torch.rand(B, (R + 1) if R else 1, 2 * K, device=dev) * 0.8 + 0.1) * H
        x = torch.rand(B, T, 3, H, H, device=dev)
        tmpl = torch.randn(K * h * h, device=dev)
        cont = torch.randn(K * 3 * h * h, device=dev)
        bg = torch.rand(3 * H * H, device=dev)
        w = torch.zeros(B, max(R, 1), device=dev)
        w[:, :live if R else 1] = 1.0 / (F * fr)
        out = torch.empty(F * fr, device=dev)
        sse = torch.empty(F, device=dev)
        if R:
            pv = (pos.data_ptr() + 2 * K * 4, (R + 1) * 2 * K, 2 * K, R)
            tv = (x.data_ptr() + 4 * fr * 4, T * fr, R, fr)
        else:
            pv = (pos.data_ptr(), 0, 2 * K, 0)
            tv = (x.data_ptr(), fr, 0, 0)
        slab_len = int(L.paig_decoder_slab_len(K, h, H))
        nb = L.paig_decoder_bwd_blocks(F, R, live, K, h, H)
        slab = torch.empty(nb * slab_len, device=dev)
        scr = L.paig_decoder_bwd_scratch(F, K, h, H)
        scratch = torch.empty(scr, device=dev) if scr else None
        dpos = torch.empty(F * 2 * K, device=dev)

        def fwd():
            L.paig_decoder_fwd(*pv, tmpl.data_ptr(), cont.data_ptr(), bg.data_ptr(), out.data_ptr(), fr, *tv,
                               sse.data_ptr(), F, K, h, H, st)

        def bwd():
            rc = L.paig_decoder_bwd(*pv, tmpl.data_ptr(), cont.data_ptr(), bg.data_ptr(), *tv, w.data_ptr(), None,
                                    fr, dpos.data_ptr(), slab.data_ptr(),
                                    None if scratch is None else scratch.data_ptr(), F, live if R else 0, K, h, H,
                                    st)
            assert rc == 0, L.paig_last_error()

        nlive = B * live if R else F
        for kind, fn, nbytes in (("fwd", fwd, 2 * F * fr * 4),
                                 ("bwd", bwd, nlive * fr * 4 + F * 2 * K * 4 + slab_len * 4)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            extra = f" slab_rows={nb} slab_MB={nb * slab_len * 4 / 1e6:.2f}" if kind == "bwd" else ""
            print(f"{name:15s} {kind} frames={F:6d} live={nlive:6d} {us:9.2f} us  alg={nbytes / 1e6:8.2f} MB "
                  f"{nbytes / us / 1e3:7.1f} GB/s frac={nbytes / us / 1e3 / 8000:.3f}{extra}", flush=True)


if __name__ == "__main__":
    main()
