"""Spatial transformer (reference nn/network/stn.py:5-23).

PhysicsNet's decoder runs its translation-only STN fused with compositing and
the loss (``paig_decoder_fwd/bwd``, csrc/decoder.hip).  The general helpers
are provided on their own kernels (``paig_stn_fwd/bwd``): any affine theta,
bilinear, zeros padding, align_corners=False, as affine_grid + grid_sample.
"""
from paig_reproduction_amd.nn.network.native_modules import stn, batch_transformer  # noqa: F401
