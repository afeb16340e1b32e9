"""CPU checks of the C-ABI boundary: the library builds/loads, exports every
symbol include/paig_hip.h declares, and the ctypes table in _lib.py matches
the header prototypes argument by argument (no compute: no GPU here)."""
import ctypes
import os
import re

import pytest

from paig_reproduction_amd import _lib

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

CMAP = {"int": _lib.I, "long long": _lib.LL, "float": _lib.F32, "double": _lib.F64, "size_t": _lib.SZ}


def header_protos():
    h = open(os.path.join(REPO, "include", "paig_hip.h")).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    out = {}
    for m in re.finditer(r"([\w\s\*]+?)\b(paig_\w+)\s*\(([^)]*)\)\s*;", h):
        args = [a.strip() for a in m.group(3).split(",")] if m.group(3).strip() not in ("", "void") else []
        types = []
        for a in args:
            t = re.sub(r"\b\w+$", "", a).strip()  # drop the parameter name
            t = t.replace("const ", "").strip()
            types.append("ptr" if "*" in t or t.endswith("_fn") else t)   # (callback typedefs: pointers)
        out[m.group(2)] = types
    return out


def test_header_matches_ctypes_table():
    protos = header_protos()
    assert set(protos) == set(_lib.SIGNATURES), set(protos) ^ set(_lib.SIGNATURES)
    for name, types in protos.items():
        argtypes = _lib.SIGNATURES[name][1]
        assert len(types) == len(argtypes), name
        for i, (t, a) in enumerate(zip(types, argtypes)):
            want = _lib.P if t == "ptr" else CMAP[t]
            assert a is want, f"{name} arg {i}: header {t} vs ctypes {a}"


def test_library_loads_and_exports_every_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libpaig_hip.so is not built (run __graft_entry__.build())")
    dll = ctypes.CDLL(_lib.LIB_PATH)
    for name in header_protos():
        assert hasattr(dll, name), name
    L = _lib.lib()
    assert L.paig_abi_version() == _lib.ABI_VERSION
    # size queries are host-only and safe without a GPU
    assert L.paig_decoder_slab_len(2, 16, 32) == 2 * 16 * 16 * 4 + 3 * 32 * 32
    assert L.paig_decoder_bwd_blocks(1600, 0, 0, 2, 16, 32) >= 1
    # live rollout frames only: 100 sequences x 6 of 46 steps, >= 3 frames per block
    # (unless PAIG_DEC_FPB_MIN overrides it)
    fmin = max(1, int(os.environ.get("PAIG_DEC_FPB_MIN", "3")))
    assert L.paig_decoder_bwd_blocks(4600, 46, 6, 2, 16, 32) == -(-600 // max(fmin, 3))
    assert L.paig_vfn_bwd_blocks(3072) == 384
    # the U-Net plan facts the engine reads (csrc/unet.hip is the one plan):
    # convs, buffers, the 1x1 head's input buffer and width
    assert [L.paig_unet_query(0, 2, w) for w in range(5)] == [13, 16, 14, 8, 15]   # ShallowUNet: c13 on A12
    assert [L.paig_unet_query(1, 2, w) for w in range(5)] == [18, 22, 20, 16, 21]  # UNet: c18 on A17
    # the head input fills its buffer from channel 0 (the fused head kernels' contract)
    assert [L.paig_unet_query(n, 2, w) for n in (0, 1) for w in (5, 6)] == [0, 8, 0, 16]
    # workspace layouts: inference holds no gradients; a head-input gradient exists for training
    for net, H in ((0, 32), (1, 64)):
        full = L.paig_unet_workspace_ex(net, 10, H, 2, 128, 1)
        assert 0 < L.paig_unet_workspace_ex(net, 10, H, 2, 128, 1 | 4) < full
        hb = L.paig_unet_query(net, 2, 2)
        assert 0 <= L.paig_unet_buffer(net, 10, H, 2, 128, 1, 1, hb) < full
        assert L.paig_unet_buffer(net, 10, H, 2, 128, 1 | 4, 1, hb) == -1


def test_product_path_refuses_cpu_tensors():
    import torch
    with pytest.raises(_lib.PaigError):
        _lib.require_device(torch.zeros(3))
