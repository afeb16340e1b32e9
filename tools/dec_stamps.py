"""Phase timeline of the decoder backward from the s_memtime stamps of the
diagnostic build (tools/dec_stamps.sh; PAIG_AB_LIB=.../diag/libpaig_stamps.so).

usage: PAIG_AB_LIB=paig_reproduction_amd/csrc/diag/libpaig_stamps.so python tools/dec_stamps.py [case]
Per iteration (averaged over blocks 0-3 and their waves): cycles from the
loop top to the end of pass 2, of pass 1, of the tables, to the barrier's
release; and the spread (max - min) of the waves' barrier arrivals.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "spring_roll"
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import dec_bench
    sys.argv = ["dec_bench.py", "1", case]
    dec_bench.main()   # in this process: the stamps stay in its device memory
    so = ctypes.CDLL(os.environ["PAIG_AB_LIB"])
    buf = np.zeros((4, 16, 33, 6), dtype=np.uint64)
    torch.cuda.synchronize()
    rc = so.paig_dec_stamps_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    assert rc == 0, rc
    b = buf.astype(np.int64)
    names = ["top->pass2 end", "pass2->pass1 end", "pass1->tables end", "tables->barrier out"]
    for blk in range(4):
        valid = [it for it in range(1, 33) if (b[blk, :, it, 1] > 0).all() and (b[blk, :, it, 5] > 0).all()]
        if not valid:
            continue
        print(f"block {blk}: prologue->loop {np.mean(b[blk, :, 1, 1] - b[blk, :, 0, 0]):.0f} cyc (iteration 0 incl.)")
        for it in valid[:8]:
            w = b[blk, :, it]
            seg = [w[:, 2] - w[:, 1], w[:, 3] - w[:, 2], w[:, 4] - w[:, 3], w[:, 5] - w[:, 4]]
            arr = w[:, 4]
            print(f"  it {it:2d}: " + "  ".join(f"{n} {np.mean(x):6.0f} (max {np.max(x):6.0f})" for n, x in zip(names, seg))
                  + f"  arrival spread {arr.max() - arr.min():6.0f}  total {np.mean(w[:, 5] - w[:, 1]):6.0f}")
        # per wave, relative to the earliest loop-top stamp of the iteration
        for it in valid[2:4]:
            w = b[blk, :, it]
            t0 = w[:, 1].min()
            print(f"  it {it} per wave (cycles from the first wave's loop top): top / pass2 end / pass1 end / "
                  "tables end / barrier in / out")
            for wv in range(w.shape[0]):
                print("    w%2d " % wv + " ".join("%6d" % (w[wv, ph] - t0) for ph in range(1, 6)))


if __name__ == "__main__":
    main()
