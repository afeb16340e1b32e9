"""Per-launch timing of the localiser's dense tail (paig_gemm_parts +
paig_dense_tail_fwd, paig_head_l2_bwd) at the spring B=100 shape, HIP events
around back-to-back launches.  usage: python tools/tail_bench.py [reps] [KF]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paig_reproduction_amd._lib import lib  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    KF = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    K, IN, n1 = 2, 200, 3072
    F = KF // K
    L = lib()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev) * 0.05
    X, W1, b1, W2, b2, W3, b3 = r(KF, n1), r(IN, n1), r(IN), r(IN, IN), r(IN), r(2, IN), r(2)
    h1, h2, h3, pos = (torch.empty(KF, IN, device=dev), torch.empty(KF, IN, device=dev),
                       torch.empty(KF, 2, device=dev), torch.empty(F, 2 * K, device=dev))
    nparts = L.paig_gemm_parts_size(KF, IN, n1, 6)
    part = torch.empty(nparts, device=dev)
    S = [0]

    def gemm():
        S[0] = L.paig_gemm_parts(0, 1, KF, IN, n1, X.data_ptr(), n1, W1.data_ptr(), n1, part.data_ptr(), nparts, 6, st)

    w2t = W2.t().contiguous()   # as paig_conv_wprep's dg = 2 job leaves it

    def tail():
        L.paig_dense_tail_fwd(part.data_ptr(), S[0], b1.data_ptr(), h1.data_ptr(), None, w2t.data_ptr(),
                              b2.data_ptr(),
                              h2.data_ptr(), W3.data_ptr(), b3.data_ptr(), h3.data_ptr(), pos.data_ptr(), F, K, IN,
                              float(16.0), st)
    print("gemm_parts  %.2f us (S=%d)" % (timeit(gemm, reps), S[0]))
    print("tail_fwd    %.2f us" % timeit(tail, reps))
    dpos = r(F, 2 * K)
    dh2, dh1 = torch.empty(KF, IN, device=dev), torch.empty(KF, IN, device=dev)
    nb = L.paig_head_bwd_blocks(KF)
    slab = torch.empty(nb * (2 * IN + 2), device=dev)
    nul = [None] * 11

    def bwd():
        L.paig_head_l2_bwd(h2.data_ptr(), h3.data_ptr(), dpos.data_ptr(), W3.data_ptr(), dh2.data_ptr(),
                           slab.data_ptr(), F, K, IN, 16.0, None, None, 0, 0, 0, 0, W2.data_ptr(), h1.data_ptr(),
                           dh1.data_ptr(), 0, *nul, st)

    def bwd_old():
        L.paig_head_bwd(h2.data_ptr(), h3.data_ptr(), dpos.data_ptr(), W3.data_ptr(), dh2.data_ptr(),
                        slab.data_ptr(), F, K, IN, 16.0, st)
    print("head_l2_bwd %.2f us" % timeit(bwd, reps))
    print("head_bwd    %.2f us" % timeit(bwd_old, reps))


if __name__ == "__main__":
    main()
