"""ctypes binding of libpaig_hip.so (the C ABI declared in include/paig_hip.h).

The library is built in-tree (``make -C paig_reproduction_amd/csrc`` or
``__graft_entry__.build()``).  There is deliberately no fallback: if the
library cannot be loaded, every product call raises.
"""
import ctypes
import os

import torch  # noqa: F401  (loads torch's HIP runtime first; the .so binds to it)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpaig_hip.so")
# A/B tooling only (tools/conv_bench.py against an older build): another .so
# slots per conv of paig_conv2d_fwd_ex / paig_conv2d_wgrad_ex (PAIG_XMAX_SLOTS)
XMAX_SLOTS = 2048

AB_PATH = os.environ.get("PAIG_AB_LIB")
# include/paig_hip.h PAIG_ABI_VERSION: the SIGNATURES below are this version's
ABI_VERSION = 8

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F32 = ctypes.c_float
F64 = ctypes.c_double
SZ = ctypes.c_size_t

# name -> (restype, argtypes); must mirror include/paig_hip.h exactly
SIGNATURES = {
    "paig_last_error": (ctypes.c_char_p, []),
    "paig_abi_version": (I, []),
    "paig_f16_range_status": (I, [I]),
    "paig_conv2d_fwd": (I, [P, LL, I, LL, P, LL, P, LL, P, P, I, I, I, I, I, I, I, P]),
    "paig_conv2d_wgrad": (I, [P, LL, I, LL, P, LL, P, I, P, I, I, I, I, I, I, I, P]),
    "paig_conv2d_fwd_ex": (I, [P, LL, I, LL, P, LL, P, LL, P, P, I, I, I, I, I, I, I, P, I, P]),
    "paig_conv2d_fwd_pw": (I, [P, LL, I, LL, P, LL, P, LL, P, P, I, I, I, I, I, I, I, P, I, P, LL, P, P]),
    "paig_conv_wprep_size": (LL, [I, I, I]),
    "paig_conv_wprep": (I, [I, P, P, P, P, P, P, P]),
    "paig_conv_wprep_defer": (I, [I, P, P, P, P, P, P, P]),
    "paig_conv_wprep_flush": (I, [P]),
    "paig_conv2d_wgrad_ex": (I, [P, LL, I, LL, P, LL, P, I, P, I, I, I, I, I, I, I, P, I, P]),
    "paig_conv2d_wgrad_pf": (I, [P, LL, I, LL, P, LL, P, LL, P, LL, P, I, P, I, I, I, I, I, I, I, P, I, P]),
    "paig_conv2d_mfma_supported": (I, [I, I, I, I, I, I, I]),
    "paig_debug_fwd_block_cap": (I, [I]),
    "paig_conv2d_bwd_supported": (I, [I, I, I, I, I, I]),
    "paig_conv2d_bwd": (I, [P, LL, I, LL, P, LL, P, LL, P, LL, P, P, I, P, I, I, I, I, I, I, I, P, I, P, LL, P, LL,
                            P, P]),
    "paig_conv2d_fwd_pwc": (I, [P, LL, I, LL, P, LL, P, LL, P, P, I, I, I, I, I, I, I, P, I, P, LL, P, LL, P, P]),
    "paig_gather_u8_f32": (I, [P, P, P, I, LL, P]),
    "paig_gather_u8_f32_ex": (I, [P, P, P, I, LL, LL, P, P]),
    "paig_velmlp_fwd": (I, [P, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P]),
    "paig_velmlp_vfn_fwd": (I, [P, I, I, I, I, P, P, P, P, P, P, P, P, P, P, I, P, P, P, P, P, P, P, P, P]),
    "paig_velmlp_bwd_blocks": (I, [I]),
    "paig_velmlp_slab_len": (I, [I]),
    "paig_velmlp_bwd": (I, [P, P, P, P, P, P, P, P, P, I, I, P]),
    "paig_head_fwd": (I, [P, P, P, P, P, I, I, I, F32, P]),
    "paig_dense_tail_fwd": (I, [P, I, P, P, P, P, P, P, P, P, P, P, I, I, I, F32, P]),
    "paig_head_l2_bwd": (I, [P, P, P, P, P, P, I, I, I, F32, P, P, I, I, I, I, P, P, P, I, P, P, P, P, P, P, P, P, P,
                             P, P, P]),
    "paig_head_bwd_blocks": (I, [I]),
    "paig_head_l2_bwd_blocks": (I, [I]),
    "paig_head_bwd": (I, [P, P, P, P, P, P, I, I, I, F32, P]),
    "paig_head_bwd_vel": (I, [P, P, P, P, P, P, I, I, I, F32, P, P, I, I, I, I, P]),
    "paig_head_bwd_vel_vfn2": (I, [P, P, P, P, P, P, I, I, I, F32, P, P, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P,
                                   P]),
    "paig_unet_workspace": (SZ, [I, I, I, I, I]),
    "paig_localiser_workspace": (SZ, [I, I, I, I, I]),
    "paig_localiser_fwd": (I, [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, F32, I, P, SZ, P]),
    "paig_localiser_bwd": (I, [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, F32, I, P, SZ, P]),
    "paig_velmlp_rollout_fwd": (I, [I, P, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, P]),
    "paig_velmlp_rollout_bwd_workspace": (SZ, [I, I, I]),
    "paig_velmlp_rollout_bwd": (I, [I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P, SZ, P]),
    "paig_unet_fwd": (I, [I, I, I, I, I, P, LL, I, LL, P, P, P, P, SZ, P]),
    "paig_unet_bwd": (I, [I, I, I, I, I, P, LL, I, LL, P, P, P, P, P, SZ, P]),
    "paig_unet_workspace_ex": (SZ, [I, I, I, I, I, I]),
    "paig_unet_buffer": (LL, [I, I, I, I, I, I, I, I]),
    "paig_unet_query": (I, [I, I, I]),
    "paig_unet_fwd_ex": (I, [I, I, I, I, I, I, P, LL, I, LL, P, P, P, P, P, P, SZ, P, P, P]),
    "paig_unet_bwd_ex": (I, [I, I, I, I, I, I, P, LL, I, LL, P, P, P, P, I, P, P, P, P, P, P, SZ, P, P, P]),
    "paig_maxpool2_fwd": (I, [P, LL, P, LL, I, I, I, I, P]),
    "paig_maxpool2_fwd_codes": (I, [P, LL, P, LL, P, LL, I, I, I, I, P]),
    "paig_maxpool2_bwd_relu": (I, [P, LL, P, LL, P, LL, I, I, I, I, P]),
    "paig_upsample2_fwd": (I, [P, LL, P, LL, I, I, I, I, I, I, P]),
    "paig_upsample2_bwd": (I, [P, LL, P, LL, P, LL, I, I, I, I, I, I, I, P]),
    "paig_mask_softmax_fwd": (I, [P, P, LL, I, LL, P, P, P, I, I, I, I, I, P]),
    "paig_mask_softmax_bwd": (I, [P, P, LL, I, LL, P, P, P, I, I, I, I, I, I, P]),
    "paig_head_mask_blocks": (I, [I, I, I]),
    "paig_head_mask_fwd": (I, [P, P, P, P, LL, I, LL, P, P, I, I, I, I, P]),
    "paig_head_mask_bwd": (I, [P, P, P, P, LL, I, LL, P, P, P, P, I, I, I, I, P]),
    "paig_head_mask_fwd_ex": (I, [P, P, P, P, LL, I, LL, P, P, P, I, I, I, I, I, I, P]),
    "paig_head_mask_bwd_ex": (I, [P, P, P, P, LL, I, LL, P, P, P, P, I, I, I, I, I, I, P]),
    "paig_pos_head_fwd": (I, [P, P, I, I, F32, P]),
    "paig_pos_head_bwd": (I, [P, P, P, I, I, F32, P]),
    "paig_gemm_workspace": (SZ, [I, I, I]),
    "paig_gemm_parts_size": (SZ, [I, I, I, I]),
    "paig_gemm_parts": (I, [I, I, I, I, I, P, LL, P, LL, P, SZ, I, P]),
    "paig_gemm_defer_epilogue": (I, [I]),
    "paig_gemm_flush": (I, [P]),
    "paig_gemm": (I, [I, I, I, I, I, F32, P, LL, P, LL, F32, P, LL, P, I, I, P, LL, P, P, SZ, P]),
    "paig_gemm_ex": (I, [I, I, I, I, I, F32, P, LL, P, LL, F32, P, LL, P, I, I, P, LL, P, P, SZ, I, P]),
    "paig_colsum_workspace": (SZ, [I, I]),
    "paig_colsum": (I, [P, I, I, LL, P, I, P, P]),
    "paig_slab_reduce": (I, [P, I, LL, I, P, I, P]),
    "paig_slab_reduce_multi": (I, [I, P, P, P, P, I, P]),
    "paig_axpby": (I, [P, P, LL, F32, F32, P]),
    "paig_vfn_fwd": (I, [P, P, P, P, P, P, P, I, P]),
    "paig_vfn_bwd_blocks": (I, [I]),
    "paig_vfn_bwd": (I, [P, P, I, P, P, P, P, P, P, P, I, P]),
    "paig_vfn_fwd_multi": (I, [I, P, P, P, P, P, P, P, P, P]),
    "paig_vfn_bwd_multi": (I, [I, P, P, P, P, P, P, P, P, P, P, P, P]),
    "paig_vfn_bwd1_multi": (I, [I, P, P, P, P, P, P, P, P, P, P, P, P]),
    "paig_vel_pack": (I, [P, P, I, I, I, I, I, P]),
    "paig_vel_unpack_add": (I, [P, P, P, I, I, I, I, I, P]),
    "paig_rollout_fwd": (I, [I, P, LL, P, P, P, P, P, I, I, I, P]),
    "paig_rollout_bwd_blocks": (I, [I]),
    "paig_rollout_bwd": (I, [I, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, P]),
    "paig_decoder_fwd": (I, [P, LL, LL, I, P, P, P, P, LL, P, LL, I, LL, P, I, I, I, I, P]),
    "paig_decoder_fwd_rollout": (I, [I, P, LL, P, P, P, P, P, I, I, I, P, LL, LL, I, P, P, P, P, LL, P, LL, I, LL, P, I, I,
                                      I, I, P]),
    "paig_decoder_fwd_t8": (I, [P, LL, LL, I, P, P, P, P, LL, P, P, LL, I, LL, P, I, I, I, I, P]),
    "paig_decoder_bwd_blocks": (I, [I, I, I, I, I, I]),
    "paig_decoder_slab_len": (SZ, [I, I, I]),
    "paig_decoder_bwd_scratch": (SZ, [I, I, I, I]),
    "paig_decoder_bwd": (I, [P, LL, LL, I, P, P, P, P, LL, I, LL, P, P, LL, P, P, P, I, I, I, I, I, P]),
    "paig_decoder_bwd_ex": (I, [P, LL, LL, I, P, P, P, P, P, P, LL, I, LL, P, I, P, P, P, F32, I, I, I, I, P, LL, P, P, P,
                                 I, I, I, I, I, P]),
    "paig_decoder_bwd_t8": (I, [P, LL, LL, I, P, P, P, P, P, LL, I, LL, P, P, LL, P, P, P, I, I, I, I, I, P]),
    "paig_decoder_parts": (I, [P, LL, P, P, P, P, P, I, I, I, I, P]),
    "paig_stn_fwd": (I, [P, P, P, I, I, I, I, I, I, P]),
    "paig_stn_bwd": (I, [P, P, P, P, P, I, I, I, I, I, I, P]),
    "paig_stn_fwd_f64": (I, [P, P, P, I, I, I, I, I, I, P]),
    "paig_stn_bwd_f64": (I, [P, P, P, P, P, I, I, I, I, I, I, P]),
    "paig_relu_mask": (I, [P, P, LL, P]),
    "paig_loss_reduce": (I, [P, P, I, I, I, I, F32, P, P, P, P]),
    "paig_loss_bwd": (I, [P, P, P, F32, P, P, I, I, I, I, P]),
    "paig_frame_sse": (I, [P, LL, I, LL, P, LL, I, LL, P, I, I, P]),
    "paig_frame_sse_bwd": (I, [P, LL, I, LL, P, LL, I, LL, P, P, I, I, P]),
    "paig_rmsprop_f32": (I, [P, P, P, LL, F32, F32, F32, P]),
    "paig_rmsprop_f64": (I, [P, P, P, LL, F64, F64, F64, P]),
    "paig_rmsprop_mixed": (I, [P, P, P, LL, P, P, P, LL, F64, F64, F64, P]),
    "paig_adam_f32": (I, [P, P, P, P, LL, F32, F32, F32, F32, F32, F32, P]),
    "paig_adam_f64": (I, [P, P, P, P, LL, F64, F64, F64, F64, F64, F64, P]),
    "paig_sgd_f32": (I, [P, P, P, LL, F32, F32, I, P]),
    "paig_sgd_f64": (I, [P, P, P, LL, F64, F64, I, P]),
}

_QUERY = {"paig_last_error", "paig_abi_version", "paig_f16_range_status", "paig_conv2d_mfma_supported",
          "paig_debug_fwd_block_cap",
          "paig_conv2d_bwd_supported", "paig_velmlp_bwd_blocks",
          "paig_velmlp_slab_len", "paig_head_bwd_blocks", "paig_head_l2_bwd_blocks", "paig_head_mask_blocks", "paig_conv_wprep_size", "paig_gemm_workspace", "paig_colsum_workspace",
          "paig_gemm_parts_size", "paig_gemm_parts", "paig_unet_workspace", "paig_unet_workspace_ex",
          "paig_unet_buffer", "paig_unet_query", "paig_localiser_workspace",
          "paig_velmlp_rollout_bwd_workspace",
          "paig_vfn_bwd_blocks", "paig_rollout_bwd_blocks", "paig_decoder_bwd_blocks", "paig_decoder_slab_len",
          "paig_decoder_bwd_scratch"}


class PaigError(RuntimeError):
    pass


class _Lib:
    def __init__(self, path=LIB_PATH):
        if not os.path.exists(path):
            raise PaigError(f"libpaig_hip.so not built at {path}: run `make -C paig_reproduction_amd/csrc` "
                            "(or __graft_entry__.build()); there is no CPU fallback")
        self.path = path
        self.dll = ctypes.CDLL(path)
        self.dll.paig_abi_version.restype = I
        self.dll.paig_abi_version.argtypes = []
        ver = self.dll.paig_abi_version()
        if ver != ABI_VERSION:
            # an A/B build of another interface version would take this
            # version's argument lists (shifted arguments, misread layouts)
            raise PaigError(f"{path}: C ABI version {ver}, this binding is version {ABI_VERSION}")
        self.fns = {}
        for name, (rt, args) in SIGNATURES.items():
            if path != LIB_PATH and not hasattr(self.dll, name):
                continue   # an older A/B build
            f = getattr(self.dll, name)
            f.restype = rt
            f.argtypes = args
            self.fns[name] = f

    def __getattr__(self, name):
        fns = self.__dict__.get("fns")
        if fns is None or name not in fns:
            raise AttributeError(name)
        f = fns[name]
        if name in _QUERY:
            return f

        def call(*a):
            rc = f(*a)
            if rc != 0:
                msg = self.fns["paig_last_error"]().decode(errors="replace")
                raise PaigError(f"{name} failed (rc={rc}): {msg}")
            return rc

        call.__name__ = name
        return call


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _Lib(AB_PATH or LIB_PATH)
    return _lib


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_handle(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def require_device(t):
    if not (torch.is_tensor(t) and t.is_cuda):
        raise PaigError("paig_reproduction_amd runs only on a HIP device (MI355X); got a "
                        f"{'CPU' if torch.is_tensor(t) else type(t).__name__} tensor. There is no CPU fallback.")
