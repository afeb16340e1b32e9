"""Per-launch timing and accuracy of the pre-split dense GEMM (paig_ps_split +
paig_psgemm) at the train step's dense-layer shapes, beside paig_gemm_ex math 6.

usage: python tools/psgemm_bench.py [reps=50] [rows=2000]
(PAIG_PS_TILE=0..3 in the environment picks the wave tile.)  Prints per shape:
split time (both operands, one launch), psgemm time (split-K epilogue
included), the old GEMM's time, and the max error of both vs float64 relative
to max |C|.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paig_reproduction_amd._lib import lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    L = lib()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(0)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    for (I, O) in ((3072, 200), (200, 200)):
        x = torch.rand(rows, I, generator=g).to(dev)
        W = (torch.randn(O, I, generator=g) * 0.05).to(dev)
        dy = (torch.randn(rows, O, generator=g) * 1e-3).to(dev)
        # (name, M, N, K, A op (src, sr, sk), B op, ref, old-gemm args (ta, tb, A, lda, B, ldb))
        cases = [
            ("fwd", rows, O, I, (x, I, 1), (W, I, 1), x.double() @ W.double().T, (0, 1, x, I, W, I)),
            ("dgrad", rows, I, O, (dy, O, 1), (W, 1, I), dy.double() @ W.double(), (0, 0, dy, O, W, I)),
            ("wgrad", O, I, rows, (dy, 1, O), (x, 1, I), dy.double().T @ x.double(), (1, 0, dy, O, x, I)),
        ]
        for name, M, N, K, a, b, ref, old in cases:
            ia = torch.empty(L.paig_ps_bytes(M, K) // 4 + 64, device=dev)
            ib = torch.empty(L.paig_ps_bytes(N, K) // 4 + 64, device=dev)
            C = torch.empty(M, N, device=dev)
            ws = torch.empty(max(1, L.paig_psgemm_workspace(M, N, K), L.paig_gemm_workspace(M, N, K)), device=dev)
            srcs = (ctypes.c_void_p * 2)(a[0].data_ptr(), b[0].data_ptr())
            srs = (ctypes.c_longlong * 2)(a[1], b[1])
            sks = (ctypes.c_longlong * 2)(a[2], b[2])
            Rs = (ctypes.c_int * 2)(M, N)
            Ks = (ctypes.c_int * 2)(K, K)
            dsts = (ctypes.c_void_p * 2)(ia.data_ptr(), ib.data_ptr())

            def split():
                L.paig_ps_split(2, srcs, srs, sks, Rs, Ks, dsts, None, st)

            def gemm():
                L.paig_psgemm(M, N, K, ia.data_ptr(), ib.data_ptr(), 1.0, C.data_ptr(), N, 0.0, None, 0, 0, None, 0,
                              ws.data_ptr(), ws.numel(), st)

            def oldg():
                ta, tb, A_, lda, B_, ldb = old
                L.paig_gemm_ex(ta, tb, M, N, K, 1.0, A_.data_ptr(), lda, B_.data_ptr(), ldb, 0.0, C.data_ptr(), N,
                               None, 0, 0, None, 0, None, ws.data_ptr(), ws.numel(), 6, st)

            t_split = timed(split)
            t_gemm = timed(gemm)
            err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
            t_old = timed(oldg)
            err_old = ((C.double() - ref).abs().max() / ref.abs().max()).item()
            byts = 4 * (M * K + K * N + M * N)
            print(f"l{1 if I > 200 else 2}_{name:6s} M={M:5d} N={N:5d} K={K:5d}  split {t_split:6.1f} us  psgemm "
                  f"{t_gemm:6.1f} us ({byts / t_gemm / 1e3:5.0f} GB/s)  old {t_old:6.1f} us   err {err:.2e} "
                  f"old {err_old:.2e}", flush=True)


if __name__ == "__main__":
    main()
