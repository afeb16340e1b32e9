"""Pre-split dense GEMM (paig_ps_split + paig_psgemm, csrc/psgemm.hip) against
float64 torch: the three forms of a dense layer (forward x W^T, data gradient
dy W, weight gradient dy^T x with the bias gradient as the image's row sums),
ragged shapes (R not a multiple of 64, K not a multiple of 32), rows of wildly
different magnitudes, the split-K path and the fused epilogue.

Bar: |C - C64| <= 1e-5 (|A| |B|)  elementwise (+1e-30): each operand keeps 22
significant bits per element (per-row exponents) and the products accumulate
in fp32, so the error is relative to the sum of the magnitudes of each dot
product's terms, whatever the rows' scales.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _L():
    from paig_reproduction_amd._lib import lib
    return lib()


def _img(M, K, dev):
    return torch.empty(_L().paig_ps_bytes(M, K) // 4 + 64, device=dev)


def _split(jobs, dev, rowsums=None):
    """jobs: [(src tensor, sr, sk, R, K)] -> images; rowsums: per job a tensor or None"""
    L = _L()
    imgs = [_img(R, K, dev) for _, _, _, R, K in jobs]
    n = len(jobs)
    rs = None if rowsums is None else (ctypes.c_void_p * n)(*[r.data_ptr() if r is not None else None for r in rowsums])
    L.paig_ps_split(n, (ctypes.c_void_p * n)(*[j[0].data_ptr() for j in jobs]),
                    (ctypes.c_longlong * n)(*[j[1] for j in jobs]), (ctypes.c_longlong * n)(*[j[2] for j in jobs]),
                    (ctypes.c_int * n)(*[j[3] for j in jobs]), (ctypes.c_int * n)(*[j[4] for j in jobs]),
                    (ctypes.c_void_p * n)(*[i.data_ptr() for i in imgs]), rs, torch.cuda.current_stream().cuda_stream)
    return imgs


def _gemm(M, N, K, ia, ib, dev, bias=None, act=0, auxm=0, aux=None, beta=0.0, C=None):
    L = _L()
    C = torch.zeros(M, N, device=dev) if C is None else C
    ws = torch.empty(max(1, L.paig_psgemm_workspace(M, N, K)), device=dev)
    L.paig_psgemm(M, N, K, ia.data_ptr(), ib.data_ptr(), 1.0, C.data_ptr(), N, beta,
                  bias.data_ptr() if bias is not None else None, act, auxm, aux.data_ptr() if aux is not None else None,
                  N, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
    return C


def _check(C, ref, A, B):
    bound = 1e-5 * (A.double().abs() @ B.double().abs()) + 1e-30
    err = (C.double() - ref).abs()
    assert torch.all(err <= bound), f"max err/bound {(err / bound).max().item():.3g}"


def _rows(R, K, g, spread):
    """R x K with row scales 10^u, u uniform in [-spread, spread]"""
    s = 10.0 ** ((torch.rand(R, 1, generator=g, dtype=torch.float64) * 2 - 1) * spread)
    return (torch.randn(R, K, generator=g, dtype=torch.float64) * s).float()


@pytest.mark.parametrize("M,N,K", [(2000, 200, 3072), (2000, 200, 200), (130, 37, 45), (64, 2, 6), (1, 70, 3100)])
@pytest.mark.parametrize("spread", [0.0, 6.0])
def test_psgemm_forward(M, N, K, spread):
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(M * 7 + N + K)
    x = _rows(M, K, g, spread).to(dev)
    W = _rows(N, K, g, spread).to(dev)
    b = torch.randn(N, generator=g).to(dev)
    ia, ib = _split([(x, K, 1, M, K), (W, K, 1, N, K)], dev)
    C = _gemm(M, N, K, ia, ib, dev)
    _check(C, x.double() @ W.double().T, x, W.T)
    # bias + ReLU epilogue
    C2 = _gemm(M, N, K, ia, ib, dev, bias=b, act=1)
    ref2 = torch.relu(x.double() @ W.double().T + b.double())
    bound = 1e-5 * (x.double().abs() @ W.double().abs().T + b.double().abs()) + 1e-30
    assert torch.all((C2.double() - ref2).abs() <= bound)


@pytest.mark.parametrize("rows,O,I", [(2000, 200, 3072), (2000, 200, 200), (77, 13, 130)])
def test_psgemm_dgrad_wgrad(rows, O, I):
    """dx = (dy W) * relu'(aux) (W^T image from the row-strided split) and
    dW = dy^T x with db = the row sums of dy^T (written by the split)"""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(rows + O + I)
    x = torch.rand(rows, I, generator=g).to(dev)
    W = (torch.randn(O, I, generator=g) * 0.05).to(dev)
    dy = _rows(rows, O, g, 3.0).to(dev)
    aux = torch.randn(rows, I, generator=g).to(dev)
    db = torch.full((O,), float("nan"), device=dev)
    idy, iwt, idyt, ixt = _split([(dy, O, 1, rows, O), (W, 1, I, I, O), (dy, 1, O, O, rows), (x, 1, I, I, rows)], dev,
                                 [None, None, db, None])
    dx = _gemm(rows, I, O, idy, iwt, dev, auxm=1, aux=aux)
    ref = (dy.double() @ W.double()) * (aux.double() > 0)
    bound = 1e-5 * (dy.double().abs() @ W.double().abs()) + 1e-30
    assert torch.all((dx.double() - ref).abs() <= bound)
    dW = _gemm(O, I, rows, idyt, ixt, dev)
    _check(dW, dy.double().T @ x.double(), dy.T, x)
    # the bias gradient: row sums of dy^T
    ref_db = dy.double().sum(0)
    assert torch.allclose(db.double(), ref_db, rtol=1e-5, atol=1e-6 * dy.double().abs().sum(0).max().item())


def test_psgemm_rows_independent_of_batch():
    """a forward row depends only on its own inputs: the first half of a batch
    gives bit-identical rows alone and inside the full batch (the data-
    parallel identity)"""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    M, N, K = 2000, 200, 3072
    x = _rows(M, K, g, 2.0).to(dev)
    W = (torch.randn(N, K, generator=g) * 0.05).to(dev)
    ia, ib = _split([(x, K, 1, M, K), (W, K, 1, N, K)], dev)
    (ih,) = _split([(x, K, 1, M // 2, K)], dev)
    full = _gemm(M, N, K, ia, ib, dev)
    half = _gemm(M // 2, N, K, ih, ib, dev)
    assert torch.equal(full[:M // 2], half)


def test_psgemm_zero_and_tiny_rows():
    """all-zero rows (exponent 0) and rows near the fp32 subnormal range"""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(9)
    M, N, K = 96, 40, 100
    x = torch.randn(M, K, generator=g)
    x[3] = 0
    x[5] *= 1e-35
    x[7] *= 1e30
    x = x.to(dev)
    W = torch.randn(N, K, generator=g).to(dev)
    ia, ib = _split([(x, K, 1, M, K), (W, K, 1, N, K)], dev)
    C = _gemm(M, N, K, ia, ib, dev)
    ref = x.double() @ W.double().T
    assert torch.all(C[3] == 0)
    rows = [i for i in range(M) if i != 5]
    _check(C[rows], ref[rows], x[rows], W.T)
    assert torch.allclose(C[5].double(), ref[5], rtol=1e-4, atol=1e-40)
