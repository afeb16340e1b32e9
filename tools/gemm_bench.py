"""Per-launch timing of paig_gemm_ex at the train step's dense-layer shapes
(HIP events around N back-to-back launches on one stream).

usage: python tools/gemm_bench.py [maths=4,6,0,3] [reps=50] [rows=2000] [shape names, e.g. l1_fwd,l1_wgrad]
Prints one line per (shape, math): microseconds per launch (split-K
epilogue included) and the rate of the compulsory operand/result bytes.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paig_reproduction_amd._lib import lib  # noqa: E402


def shapes(rows):
    # (name, ta, tb, M, N, K): encoder l1 (3072 -> 200) and l2 (200 -> 200)
    return [("l1_fwd", 0, 1, rows, 200, 3072), ("l1_dgrad", 0, 0, rows, 3072, 200), ("l1_wgrad", 1, 0, 200, 3072, rows),
            ("l2_fwd", 0, 1, rows, 200, 200), ("l2_dgrad", 0, 0, rows, 200, 200), ("l2_wgrad", 1, 0, 200, 200, rows)]


def main():
    maths = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "4,6,0,3").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    only = set(sys.argv[4].split(",")) if len(sys.argv) > 4 else None
    L = lib()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for name, ta, tb, M, N, K in shapes(rows):
        if only and name not in only:
            continue
        A = torch.randn(K, M, device=dev) if ta else torch.randn(M, K, device=dev)
        B = torch.randn(N, K, device=dev) if tb else torch.randn(K, N, device=dev)
        C = torch.empty(M, N, device=dev)
        rs = torch.empty(M, device=dev) if ta else None
        ws = torch.empty(max(1, L.paig_gemm_workspace(M, N, K)), device=dev)
        for math in maths:
            def run():
                return L.paig_gemm_ex(ta, tb, M, N, K, 1.0, A.data_ptr(), A.shape[1], B.data_ptr(), B.shape[1], 0.0,
                                      C.data_ptr(), N, None, 0, 0, None, 0, rs.data_ptr() if rs is not None else None,
                                      ws.data_ptr(), ws.numel(), math, st)
            assert run() == 0, L.paig_last_error()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            byts = 4 * (M * K + K * N + M * N)
            print(f"{name:9s} math {math} {us:8.1f} us  {byts / us / 1e3:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
